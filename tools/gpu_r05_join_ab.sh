#!/bin/bash
# Round 5: the N > 1 headline's node form over peer-mapped nodes rehearsed with N processes sharing
# the one MI355X (bench.py --child-transport node-ipc, as multi_gpu runs it): the serial join
# (EXT_MPI_AMD_JOIN_PARTS=1) against the fused pipelined one (join_fused.hip) with 2, 4 and 8 parts,
# interleaved. Each line: start_to_wait and the parts timed alone (copy-in, node legs), rank 0.
# Usage: gpu_r05_join_ab.sh [passes] [Ns] [parts list]
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05/join_ab
mkdir -p $O
port=29700
for pass in $(seq 1 ${1:-2}); do
  for N in ${2:-1 2 4}; do
    for parts in ${3:-1 4 2 8}; do
      port=$((port + 1))
      tag=n${N}_p${parts}_pass${pass}
      EXT_MPI_AMD_JOIN_PARTS=$parts timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
        --master-addr 127.0.0.1 --master-port $port bench.py --gpus $N --steps 20 --warmup 5 --child-transport node-ipc \
        --child-result $O/${tag}_r{rank}.json --child-deadline 240 > $O/${tag}.log 2>&1 || { tail -20 $O/${tag}.log; exit 1; }
      python3 -c "
import json; d=json.load(open('$O/${tag}_r0.json'))
s=20; print('N $N parts $parts pass $pass', 'join_parts', d.get('join_parts'), 'start_to_wait %.1f' % (d['wall']*1e6/s), 'copy_in %.1f' % (d['copy_in_fold_s']*1e6), 'legs %.1f' % (d['node_legs_s']*1e6), 'copy_out %.1f' % (d['copy_out_s']*1e6), 'checked', d['checked'])"
    done
  done
done
