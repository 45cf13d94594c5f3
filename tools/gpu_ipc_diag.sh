#!/bin/bash
# tools/ipc_diag.py with W processes sharing the one GPU; extra env (EXT_MPI_AMD_IPC_FUSED_MAX,
# DIAG_SIZES, DIAG_READ, ...) passes through. Usage: bash tools/gpu_ipc_diag.sh W TAG
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
W=$1
TAG=$2
pids=()
port=$((29700 + W))
for ((r = 0; r < W; r++)); do
  RANK=$r WORLD_SIZE=$W MASTER_ADDR=127.0.0.1 MASTER_PORT=$port timeout -k 10 180 python tools/ipc_diag.py \
    > gpurun_out/diag_${TAG}_r$r.json 2> gpurun_out/diag_${TAG}_r$r.err &
  pids+=($!)
done
st=0
for p in "${pids[@]}"; do wait $p || st=$?; done
echo "diag $TAG world $W rc=$st"
cat gpurun_out/diag_${TAG}_r*.json
exit $st
