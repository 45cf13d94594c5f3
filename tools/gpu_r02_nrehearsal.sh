#!/bin/bash
# N > 1 bench rehearsal on the 1-GPU box: 2 and 4 torchrun ranks sharing the one MI355X (IPC
# transport first, RCCL beside it -- RCCL refuses ranks sharing a GPU and reports its error).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for n in 2 4; do
  timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --steps 5 --warmup 2 > gpurun_out/bench_n$n.json \
    2> gpurun_out/bench_n$n.err || { echo "n=$n rc=$?"; tail -20 gpurun_out/bench_n$n.err; exit 1; }
  echo "n=$n ok"; head -c 1500 gpurun_out/bench_n$n.json; echo
done
