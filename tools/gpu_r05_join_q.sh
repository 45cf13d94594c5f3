#!/bin/bash
# Round 5: why the pipelined join is slower when processes share the GPU -- the same rehearsal at
# N = 1 (no peer: multi-stream overhead alone) and at N = 2 with more hardware queues per process.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05/join_q
mkdir -p $O
port=29800
run() {  # N parts tag [env...]
  N=$1; parts=$2; tag=$3; shift 3
  port=$((port + 1))
  env EXT_MPI_AMD_JOIN_PARTS=$parts "$@" timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
    --master-addr 127.0.0.1 --master-port $port bench.py --gpus $N --steps 20 --warmup 5 --child-transport node-ipc \
    --child-result $O/${tag}_r{rank}.json --child-deadline 240 > $O/${tag}.log 2>&1 || { tail -20 $O/${tag}.log; return 1; }
  python3 -c "
import json; d=json.load(open('$O/${tag}_r0.json'))
s=20; print('$tag', 'join_parts', d.get('join_parts'), 'start_to_wait %.1f' % (d['wall']*1e6/s), 'copy_in %.1f' % (d['copy_in_fold_s']*1e6), 'legs %.1f' % (d['node_legs_s']*1e6), 'checked', d['checked'])"
}
run 1 1 n1_p1 && run 1 4 n1_p4 && run 2 1 n2_p1_q4 && run 2 4 n2_p4_q4 && \
run 2 1 n2_p1_q16 GPU_MAX_HW_QUEUES=16 && run 2 4 n2_p4_q16 GPU_MAX_HW_QUEUES=16
