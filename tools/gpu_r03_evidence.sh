#!/bin/bash
# Round-3 closing evidence for the headline after the deferred-store schedules: PMC traffic
# (FETCH_SIZE / WRITE_SIZE, separate passes, gfx950 correction in tools/pmc_traffic.py) of the
# bench's node16 launch and of the node256 / local256 shapes, then the bench itself under
# rocprofv3 --kernel-trace --stats (its fold_kernel mean must agree with roofline.avg_launch_us).
set -u
cd "$GRAFT_REPO_ROOT"; R=$PWD; mkdir -p gpurun_out; export TMPDIR=/tmp
pass() {  # tag counter bench-args...
  local tag=$1 c=$2; shift 2
  rm -rf gpurun_out/pmc_${tag}_$c
  timeout -s KILL 150 rocprofv3 --pmc $c -d $R/gpurun_out/pmc_${tag}_$c -o run --output-format csv -- \
    python3 $R/bench.py "$@" > gpurun_out/pmc_${tag}_$c.json 2> gpurun_out/pmc_${tag}_$c.err
  local rc=$?
  echo "pmc $tag $c rc=$rc"
  [ $rc -ne 0 ] && { tail -3 gpurun_out/pmc_${tag}_$c.err; exit $rc; }
  return 0
}
for c in FETCH_SIZE WRITE_SIZE; do pass node16 $c --no-extras --no-cpu-baseline --steps 10 --warmup 2; done
python3 tools/pmc_traffic.py gpurun_out/pmc_node16_FETCH_SIZE gpurun_out/pmc_node16_WRITE_SIZE gpurun_out/traffic_node_r8_16mib_float.json node_r8_16mib_float || exit 1
for c in FETCH_SIZE WRITE_SIZE; do pass node256 $c --shape node256; done
python3 tools/pmc_traffic.py gpurun_out/pmc_node256_FETCH_SIZE gpurun_out/pmc_node256_WRITE_SIZE gpurun_out/traffic_node_r8_256mib_float.json node_r8_256mib_float || exit 1
for c in FETCH_SIZE WRITE_SIZE; do pass local256 $c --shape local256; done
python3 tools/pmc_traffic.py gpurun_out/pmc_local256_FETCH_SIZE gpurun_out/pmc_local256_WRITE_SIZE gpurun_out/traffic_local_r8_32mib_float.json local_r8_32mib_float || exit 1
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- \
  python3 $R/bench.py --no-cpu-baseline --no-extras > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || exit $?
cat gpurun_out/bench_prof.json
f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1); grep -E "fold_(deferred_)?kernel<" "$f"
t=$(find gpurun_out/prof -name "*kernel_trace.csv" | head -1); python3 tools/prof_dispatches.py "$t" "fold_(deferred_)?kernel<" 5 > gpurun_out/bench_dispatches.txt
cat gpurun_out/bench_dispatches.txt
exit 0
