#!/bin/bash
# Round evidence for the headline: smoke, bench (all extras, CPU baseline), rocprofv3 kernel
# statistics of the same bench command (fold_kernel average must agree with roofline.avg_launch_us).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
cat gpurun_out/bench.json
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extras > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || exit $?
grep fold_kernel gpurun_out/prof/run_kernel_stats.csv
cat gpurun_out/bench_prof.json
exit 0
