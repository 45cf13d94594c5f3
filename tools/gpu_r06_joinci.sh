#!/bin/bash
# Round 6: the fused node join's copy-in tile (EXT_MPI_AMD_JOIN_CI_U = vectors
# per lane and leaf of a 1024-lane tile: 2, 3, 4). Bitwise first (node-IPC tests at CI_U 4), then the
# copy-in alone (bench.py --shape joinci) and the whole Start with N processes sharing the GPU
# (bench.py --child-transport node-ipc, as tools/gpu_r05_join_sweep.sh). One line per run.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06/joinci${TAG:+_$TAG}
mkdir -p $O
CIUS=${CIUS:-2 3 4}
TESTU=${TESTU:-4}
EXT_MPI_AMD_JOIN_CI_U=$TESTU timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_node_ipc.py -k "${TESTK:-serial_and_pipelined and (fused3 or fused4) or over_peer_mapped}" > $O/tests_ciu$TESTU.log 2>&1
rc=$?; tail -n 3 $O/tests_ciu$TESTU.log; [ $rc -ne 0 ] && exit $rc
for p in 2 4; do for u in $CIUS; do
  EXT_MPI_AMD_JOIN_PARTS=$p EXT_MPI_AMD_JOIN_CI_U=$u timeout -k 10 240 python3 bench.py --shape joinci > $O/joinci_p${p}_u$u.json 2> $O/joinci_p${p}_u$u.err || { tail -5 $O/joinci_p${p}_u$u.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/joinci_p${p}_u$u.json').read())
print('joinci p$p u$u fused', d['fused']['avg_launch_us'], 'us', d['fused']['achieved_gbps'], 'GB/s | serial', d['serial']['avg_launch_us'])" | tee -a $O/summary.txt
done; done
port=29900
run() {  # N parts ciu
  port=$((port + 1))
  tag=n$1_p$2_u$3
  EXT_MPI_AMD_JOIN_PARTS=$2 EXT_MPI_AMD_JOIN_CI_U=$3 timeout -k 10 150 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 --master-port $port bench.py --gpus $1 --steps 20 --warmup 5 \
    --child-transport node-ipc --child-result $O/${tag}_r{rank}.json --child-deadline 120 > $O/${tag}.log 2>&1 || { echo "$tag failed"; tail -5 $O/${tag}.log; return 1; }
  python3 -c "
import json; d=json.load(open('$O/${tag}_r0.json'))
print('$tag', 'start_to_wait %.1f' % (d['wall']*1e6/20), 'copy_in %.1f' % (d['copy_in_fold_s']*1e6), 'legs %.1f' % (d['node_legs_s']*1e6), 'checked', d['checked'])" | tee -a $O/summary.txt
}
for N in 1 2 4; do
  run $N 1 2 || exit 1
  for c in ${RUNS:-2:2 2:3 2:4 4:4 4:2}; do IFS=: read -r p u <<< "$c"; run $N $p $u || exit 1; done
done
exit 0
