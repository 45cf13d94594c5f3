#!/bin/bash
# Round-3 closing check: the driver's GPU suite command, then smoke().
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread --durations=15 > gpurun_out/r03_full_gpu.log 2>&1
rc=$?
tail -25 gpurun_out/r03_full_gpu.log
[ $rc -ne 0 ] && { echo "GPU SUITE rc=$rc"; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03_smoke.log 2>&1; rc=$?
tail -3 gpurun_out/r03_smoke.log
exit $rc
