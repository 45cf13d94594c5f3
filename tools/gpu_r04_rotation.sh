#!/bin/bash
# Round-4: buffer-set rotation by read reuse (bench.py rotation_sets). The send/receive rotation
# sweep (tools/setsweep.hip), then the default bench under the old rule (3 sets of 256 MiB for the
# headline) and the new one, the new one again under the kernel tracer (its summary: profiles/).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/rot4
mkdir -p $O
timeout -k 10 200 tools/setsweep 16 5 48 > $O/setsweep16.txt 2>&1 || { echo "setsweep rc=$?"; exit 1; }
cat $O/setsweep16.txt
EXT_MPI_AMD_BENCH_ROTATION=legacy timeout -k 10 400 python3 bench.py > $O/bench_legacy.json 2> $O/bench_legacy.err || { echo "legacy rc=$?"; tail -5 $O/bench_legacy.err; exit 1; }
timeout -k 10 400 python3 bench.py > $O/bench_new.json 2> $O/bench_new.err || { echo "new rc=$?"; tail -5 $O/bench_new.err; exit 1; }
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py > $O/bench_prof.json 2> $O/bench_prof.err || { echo "prof rc=$?"; tail -5 $O/bench_prof.err; exit 1; }
for f in bench_legacy bench_new bench_prof; do
  python3 -c "import json,sys; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); r=d['roofline']; e=d['extras']; print('$f', d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'], d['config'].get('buffer_sets', ''), d['data'][:160]); print('  256MiB', e.get('point_256MiB', {}).get('avg_launch_us'), 'local', e.get('local_fold_256MiB', {}).get('avg_launch_us'), 'int/long', json.dumps(e.get('config3_int_long_4MiB', {}))[:200]); print('  copy', json.dumps(e.get('copy_variants_gbps')))"
done
exit 0
