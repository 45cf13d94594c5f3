#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -4 gpurun_out/gpu_tests.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 420 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
cat gpurun_out/bench.json
MIBS="16 256" bash tools/gpu_foldbench.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-extras > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || exit $?
grep fold_kernel gpurun_out/prof/run_kernel_stats.csv
