#!/bin/bash
# Multi-GPU bench path rehearsed on the one-GPU box (ranks share the GPU: IPC runs, RCCL refuses).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for n in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --steps 10 --warmup 3 > gpurun_out/r03_bench_n$n.json 2> gpurun_out/r03_bench_n$n.err
  echo "n=$n rc=$?"
  tail -c 1500 gpurun_out/r03_bench_n$n.json
  grep -i "error\|Traceback" gpurun_out/r03_bench_n$n.err | head -5
done
