#!/bin/bash
# Round-2 round-end rehearsal: the whole GPU suite as the driver runs it, then smoke + bench +
# rocprofv3 kernel statistics of the same bench command (tools/gpu_bench_evidence.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
bash tools/gpu_bench_evidence.sh
