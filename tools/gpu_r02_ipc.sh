#!/bin/bash
# Round-2 IPC session: the placement-free node barrier. test_gpu_ipc (worlds 2, 3, 4, 8 sharing
# the one MI355X, timeout recovery included), then the latency breakdown with 2 / 4 / 8 processes.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ipc.py \
  > gpurun_out/r02_ipc_tests.log 2>&1; rc=$?
echo "ipc tests rc=$rc"; grep -E "passed|failed|PASS|FAIL|Error" gpurun_out/r02_ipc_tests.log | tail -12
[ $rc -ne 0 ] && exit $rc
for W in 2 4 8; do
  pids=()
  port=$((29600 + W))
  for ((r = 0; r < W; r++)); do
    RANK=$r WORLD_SIZE=$W LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=$port IPC_LAT_OWN_STREAM=1 \
      IPC_LAT_SIZES=8,65536,1048576,16777216 timeout -k 10 240 python tools/ipc_latency.py \
      > gpurun_out/r02_ipc_lat_w${W}_r$r.json 2> gpurun_out/r02_ipc_lat_w${W}_r$r.err &
    pids+=($!)
  done
  st=0
  for p in "${pids[@]}"; do wait $p || st=$?; done
  echo "latency world $W rc=$st"; cat gpurun_out/r02_ipc_lat_w${W}_r0.json
  [ $st -ne 0 ] && { tail -5 gpurun_out/r02_ipc_lat_w${W}_r*.err; exit $st; }
done
exit 0
