#!/bin/bash
# IPC latency breakdown (tools/ipc_latency.py) with W processes sharing the one GPU; extra env
# passes through. Usage: bash tools/gpu_ipc_lat.sh W TAG
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
W=$1
TAG=$2
pids=()
port=$((29900 + W))
for ((r = 0; r < W; r++)); do
  RANK=$r WORLD_SIZE=$W LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=$port IPC_LAT_OWN_STREAM=1 \
    IPC_LAT_SIZES=${IPC_LAT_SIZES:-8,65536,1048576,16777216} timeout -k 10 240 python tools/ipc_latency.py \
    > gpurun_out/lat_${TAG}_r$r.json 2> gpurun_out/lat_${TAG}_r$r.err &
  pids+=($!)
done
st=0
for p in "${pids[@]}"; do wait $p || st=$?; done
echo "latency $TAG world $W rc=$st"; cat gpurun_out/lat_${TAG}_r0.json
exit $st
