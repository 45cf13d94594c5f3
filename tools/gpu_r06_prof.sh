#!/bin/bash
# Round-6 closing evidence, part 2: PMC traffic (FETCH_SIZE / WRITE_SIZE, separate passes, gfx950
# correction in tools/pmc_traffic.py) of the bench's node16 launch and the node256 / local256
# shapes, then the driver's own bench command under rocprofv3 --kernel-trace --stats (its kept fold
# kernel's mean must agree with roofline.avg_launch_us). Usage: gpu_r06_prof.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"; R=$PWD; export TMPDIR=/tmp
O=gpurun_out/r06/${1:-prof}
mkdir -p $O
pass() {  # tag counter bench-args...
  local tag=$1 c=$2; shift 2
  rm -rf $O/pmc_${tag}_$c
  timeout -s KILL 200 rocprofv3 --pmc $c -d $R/$O/pmc_${tag}_$c -o run --output-format csv -- \
    python3 $R/bench.py "$@" > $O/pmc_${tag}_$c.json 2> $O/pmc_${tag}_$c.err
  local rc=$?
  echo "pmc $tag $c rc=$rc"
  [ $rc -ne 0 ] && { tail -3 $O/pmc_${tag}_$c.err; exit $rc; }
  return 0
}
for c in FETCH_SIZE WRITE_SIZE; do pass node16 $c --no-extras --no-cpu-baseline --steps 10 --warmup 2; done
python3 tools/pmc_traffic.py $O/pmc_node16_FETCH_SIZE $O/pmc_node16_WRITE_SIZE $O/traffic_node_r8_16mib_float.json node_r8_16mib_float || exit 1
for c in FETCH_SIZE WRITE_SIZE; do pass node256 $c --shape node256; done
python3 tools/pmc_traffic.py $O/pmc_node256_FETCH_SIZE $O/pmc_node256_WRITE_SIZE $O/traffic_node_r8_256mib_float.json node_r8_256mib_float || exit 1
for c in FETCH_SIZE WRITE_SIZE; do pass local256 $c --shape local256; done
python3 tools/pmc_traffic.py $O/pmc_local256_FETCH_SIZE $O/pmc_local256_WRITE_SIZE $O/traffic_local_r8_32mib_float.json local_r8_32mib_float || exit 1
rm -rf $O/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_prof.json 2> $O/bench_prof.err || exit $?
tail -c 1500 $O/bench_prof.json
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/bench_kernel_stats.csv; grep -E "fold_\w*kernel<" "$f" | head
t=$(find $O/prof -name "*kernel_trace.csv" | head -1); python3 tools/prof_dispatches.py "$t" "fold_\w*kernel<" 5 > $O/bench_dispatches.txt
head -30 $O/bench_dispatches.txt
find $O -name "*.csv" -size +4M -delete
exit 0
