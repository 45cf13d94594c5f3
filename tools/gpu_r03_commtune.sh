#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "tuned or pinned or comm_form_loopback_parity" > gpurun_out/commtune_tests.log 2>&1; rc=$?
tail -4 gpurun_out/commtune_tests.log
exit $rc
