#!/bin/bash
# Round-3 re-entry check: the driver's GPU suite, smoke(), then the default N = 1 bench.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread --durations=15 > gpurun_out/r03c_gpu.log 2>&1
rc=$?
tail -25 gpurun_out/r03c_gpu.log
[ $rc -ne 0 ] && { echo "GPU SUITE rc=$rc"; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03c_smoke.log 2>&1; rc=$?
tail -3 gpurun_out/r03c_smoke.log
[ $rc -ne 0 ] && { echo "SMOKE rc=$rc"; exit $rc; }
timeout -k 10 400 python -u bench.py > gpurun_out/r03c_bench.json 2> gpurun_out/r03c_bench.err; rc=$?
tail -c 3000 gpurun_out/r03c_bench.json
exit $rc
