#!/bin/bash
# Round-4: the N > 1 bench rehearsed with 2 processes sharing the one MI355X (the node form over
# peer-mapped nodes runs; RCCL refuses two ranks on one GPU and must be reported as a failure with
# its exit code and stderr tail), bounded as the driver's run would be.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
EXT_MPI_AMD_BENCH_DEADLINE=420 timeout -k 10 560 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 10 --warmup 3 \
  > gpurun_out/r04_bench_n2_rehearsal.json 2> gpurun_out/r04_bench_n2_rehearsal.err
rc=$?
echo "rehearsal rc=$rc"
tail -c 2500 gpurun_out/r04_bench_n2_rehearsal.json
exit $rc
