#!/bin/bash
# Full round evidence on one box: parity tests, smoke, bench (all extras), rocprofv3 kernel
# statistics of the bench, FETCH_SIZE / WRITE_SIZE passes (separate runs), kernel harness.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -4 gpurun_out/gpu_tests.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
cat gpurun_out/bench.json
B="python3 bench.py --no-cpu-baseline --no-extras"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- $B > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || exit $?
grep fold_kernel gpurun_out/prof/run_kernel_stats.csv
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- $B --steps 20 > /dev/null 2> gpurun_out/pmc_fetch.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- $B --steps 20 > /dev/null 2> gpurun_out/pmc_write.err || exit $?
python3 tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/traffic_node_r8_16mib_float.json node_r8_16mib_float
MIBS="16 256" bash tools/gpu_foldbench.sh > /dev/null 2>&1 || exit $?
grep -E "PROD|prod tmpl|b256_u2_ntls |#" gpurun_out/foldbench_*.txt
exit 0
