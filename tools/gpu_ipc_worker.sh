#!/bin/bash
# tests/ipc_worker.py with W processes sharing the one GPU (extra env passes through).
# Usage: bash tools/gpu_ipc_worker.sh W TAG
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
W=$1
TAG=$2
pids=()
port=$((29800 + W))
for ((r = 0; r < W; r++)); do
  RANK=$r WORLD_SIZE=$W LOCAL_RANK=$r MASTER_ADDR=127.0.0.1 MASTER_PORT=$port IPC_DEVICE=0 \
    EXT_MPI_AMD_BARRIER_TIMEOUT=20 timeout -k 10 240 python -u tests/ipc_worker.py \
    > gpurun_out/worker_${TAG}_r$r.log 2>&1 &
  pids+=($!)
done
st=0
for p in "${pids[@]}"; do wait $p || st=$?; done
echo "worker $TAG world $W rc=$st"
grep -h "MISMATCH\|recovery\|wrong" gpurun_out/worker_${TAG}_r*.log | head -40
exit $st
