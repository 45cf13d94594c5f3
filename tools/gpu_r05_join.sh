#!/bin/bash
# Round 5: the pipelined peer-mapped node join -- the node-IPC GPU tests (default, serial, 3 parts,
# timeout recovery), then the N = 2 / 4 shared-GPU rehearsal of the bench with the serial and the
# pipelined join.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05/join
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_node_ipc.py -x -v --timeout 400 --timeout-method thread > $O/node_ipc_tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|passed|failed|Error" $O/node_ipc_tests.log | tail -20
exit $rc
