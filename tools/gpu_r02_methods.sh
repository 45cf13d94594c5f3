#!/bin/bash
# Round-2 GPU check of the cyclic / tree copy-in methods: node form, COMM loopback, the MPI layer
# and the peer-mapped (IPC) form; logs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "methods" > gpurun_out/methods_parity.log 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_mpi_layer.py \
  -m gpu -k "multi_rank" > gpurun_out/methods_mpi.log 2>&1 &&
IPC_TEST_WORLDS=4,8 timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_ipc.py > gpurun_out/methods_ipc.log 2>&1
rc=$?
tail -5 gpurun_out/methods_*.log
exit $rc
