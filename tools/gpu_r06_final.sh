#!/bin/bash
# Round-6 closing evidence, part 1: the driver's GPU suite, smoke(), the default bench (N = 1),
# then the local fold's lease fingerprint (tools/gpu_r06_localfp.sh). Usage: gpu_r06_final.sh <tag>
cd "$GRAFT_REPO_ROOT"
tag=${1:-final}
O=gpurun_out/r06/$tag
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 400 --timeout-method thread --durations=15 > $O/gpu_tests.log 2>&1
rc=$?
tail -25 $O/gpu_tests.log
[ $rc -ne 0 ] && { echo "GPU SUITE rc=$rc"; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 - "$O/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); e = d['extras']
print('headline', d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['config'].get('fold_schedules_per_set'))
print('256', {k: e['point_256MiB'].get(k) for k in ('median_launch_us', 'min_launch_us', 'max_launch_us', 'frac_of_peak_at_median')})
print('local', {k: e['local_fold_256MiB'].get(k) for k in ('avg_launch_us', 'median_launch_us', 'min_launch_us', 'max_launch_us', 'frac_of_peak_at_median')})
print('chains', {k: (v['avg_launch_us'], v['vs_linear']) for k, v in e['radix_chains_16MiB'].items()})
print('radix vs linear', [(p['copyin'], p['bytes_per_rank'], p.get('vs_linear')) for p in e['radix_sweep_node_form']])
print('crossover', e.get('radix_crossover_node_form'))
print('int/long', {k: v['avg_launch_us'] for k, v in e['config3_int_long_4MiB'].items()})
print('host', e.get('host_buffers_pcie_inclusive'))
PY
bash tools/gpu_r06_localfp.sh $tag
