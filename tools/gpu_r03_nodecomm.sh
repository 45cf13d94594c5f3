#!/bin/bash
# Round-3: the NODE form over several nodes (loopback members) and the COMM-form loopback tests.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_node_comm.py \
  tests/test_gpu_parity.py -k "node_comm or comm_" > gpurun_out/r03_nodecomm.log 2>&1
rc=$?
tail -25 gpurun_out/r03_nodecomm.log
exit $rc
