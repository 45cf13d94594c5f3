#!/bin/bash
# Round-3: the NODE form over peer-mapped nodes (processes sharing the GPU), and the loopback
# node-comm tests beside it.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_node_ipc.py \
  > gpurun_out/nodeipc_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|NODEIPC node 0|differing|passed|failed" gpurun_out/nodeipc_tests.log | tail -60
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_node_comm.py \
  > gpurun_out/nodecomm_tests.log 2>&1; rc=$?
tail -3 gpurun_out/nodecomm_tests.log
exit $rc
