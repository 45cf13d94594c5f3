#!/bin/bash
# Round-3: the stage-out copy kernel for pinned host receive buffers -- its tests, then the host
# rates of the bench (direct, staged) and the one-rank COMM form with pinned buffers.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  -k "pinned or host" > gpurun_out/stageout_tests.log 2>&1; rc=$?
tail -3 gpurun_out/stageout_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/host_stage_bench.py > gpurun_out/stageout_hostbench.txt 2>&1; rc=$?
tail -30 gpurun_out/stageout_hostbench.txt
exit $rc
