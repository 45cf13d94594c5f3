#!/bin/bash
# Bench with the configs[0] / configs[2] points, then the IPC form with 4 processes at the
# reference's published GH200 sizes (64 KiB - 64 MiB, '6;1 -4 4').
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
cat gpurun_out/bench.json
IPC_LAT_OWN_STREAM=1 IPC_LAT_SIZES=8,65536,1048576,16777216,67108864 timeout -k 10 300 \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29561 \
  tools/ipc_latency.py > gpurun_out/ipc4.json 2> gpurun_out/ipc4.err || exit $?
cat gpurun_out/ipc4.json
