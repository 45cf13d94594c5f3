#!/bin/bash
# Round 5: the fused join (1024-lane workgroups) at N = 1, 2 and 4 (processes sharing the GPU)
# against the serial join, parts 2 and 4; EXT_MPI_AMD_JOIN_GRID = per-process workgroups before
# the shared-GPU division. One line per run.
# Usage: gpu_r05_join_sweep.sh [tag] ["N:parts:grid ..."] (default: the full sweep)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05/${1:-join_sweep2}
mkdir -p $O
port=29900
run() {  # N parts grid
  port=$((port + 1))
  tag=n$1_p$2_g$3
  EXT_MPI_AMD_JOIN_PARTS=$2 EXT_MPI_AMD_JOIN_GRID=$3 timeout -k 10 120 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 --master-port $port bench.py --gpus $1 --steps 20 --warmup 5 \
    --child-transport node-ipc --child-result $O/${tag}_r{rank}.json --child-deadline 100 > $O/${tag}.log 2>&1 || { echo "$tag failed"; tail -5 $O/${tag}.log; return 1; }
  python3 -c "
import json; d=json.load(open('$O/${tag}_r0.json'))
print('$tag', 'start_to_wait %.1f' % (d['wall']*1e6/20), 'copy_in %.1f' % (d['copy_in_fold_s']*1e6), 'legs %.1f' % (d['node_legs_s']*1e6), 'checked', d['checked'])" | tee -a $O/summary.txt
}
if [ -n "$2" ]; then
  for c in $2; do IFS=: read -r N p g <<< "$c"; run $N $p $g || exit 1; done
  exit 0
fi
for N in 1 2 4; do
  run $N 1 256 || exit 1
  for g in 256 128; do for p in 2 4; do run $N $p $g || exit 1; done; done
done
