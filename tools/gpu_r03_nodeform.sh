#!/bin/bash
# Round-3: bench.py's N > 1 node-form child run alone as a one-member RCCL job on the one GPU
# (the copy-in fold and the copy-out; no inter-node legs), to exercise its code path.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29611 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
timeout -k 10 300 python3 bench.py --child-transport node --child-result gpurun_out/r03_nodeform_w1.json --steps 20 --warmup 5 \
  > gpurun_out/r03_nodeform_w1.log 2>&1
rc=$?
tail -5 gpurun_out/r03_nodeform_w1.log
cat gpurun_out/r03_nodeform_w1.json
exit $rc
