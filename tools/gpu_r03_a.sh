#!/bin/bash
# Round-3 session A: the reworked peer-mapped set-up (no writes into caller memory, outboxes,
# collective Done), then the whole -m gpu suite in the driver's order.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread --durations=0 \
  tests/test_gpu_peer_mapped.py > gpurun_out/r03a_ipc.log 2>&1 || { echo "IPC FAILED"; tail -60 gpurun_out/r03a_ipc.log; exit 1; }
tail -25 gpurun_out/r03a_ipc.log
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests \
  --deselect tests/test_gpu_peer_mapped.py > gpurun_out/r03a_gpu.log 2>&1 || { echo "GPU SUITE FAILED"; tail -60 gpurun_out/r03a_gpu.log; exit 1; }
tail -5 gpurun_out/r03a_gpu.log
