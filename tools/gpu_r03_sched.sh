#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for k in 512 2048 32768; do
  timeout -k 10 300 tools/schedbench $k 7 10 > gpurun_out/sched_$k.txt 2>&1; echo "rc=$? chunk $k"
  cat gpurun_out/sched_$k.txt
done
