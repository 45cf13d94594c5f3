#!/bin/bash
# Round-3 session B: single-process GPU suite, the bench (N = 1), and its rocprof kernel trace.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
true && \
true

timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r03b_bench.json 2> gpurun_out/r03b_bench.err || { echo "BENCH FAILED"; tail -30 gpurun_out/r03b_bench.err; exit 1; }
cat gpurun_out/r03b_bench.json
rm -rf gpurun_out/r03b_prof
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r03b_prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/r03b_bench_prof.json 2> gpurun_out/r03b_bench_prof.err || { echo "PROF FAILED"; tail -20 gpurun_out/r03b_bench_prof.err; exit 1; }
find gpurun_out/r03b_prof -name "*kernel_stats.csv" | head -3
