#!/bin/bash
# Round 6 A/B: the fused join's copy-in load issue (EXT_MPI_AMD_JOIN_CI_LOAD: 0 source-major
# nontemporal loads, 1 buffer loads, 2 buffer loads staggered, 3 vector-major), float, 8 leaves.
# Bitwise node tests under each, the copy-in alone (bench.py --shape joinci), whole Starts N = 2, 4.
# The switch was a temporary build of join_fused.hip; buffer loads (1) were adopted and the switch
# removed, so this script now reproduces only with that build (profiles/r06/ciload/).
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06/ciload
mkdir -p $O
for v in 1 2 3; do
  EXT_MPI_AMD_JOIN_CI_LOAD=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    "tests/test_gpu_node_ipc.py::test_node_form_over_peer_mapped_nodes[2]" "tests/test_gpu_node_ipc.py::test_node_form_over_peer_mapped_nodes[4]" \
    "tests/test_gpu_node_ipc.py::test_node_join_serial_and_pipelined[2-fused3]" "tests/test_gpu_node_ipc.py::test_node_join_serial_and_pipelined[4-fused3]" > $O/tests_v$v.log 2>&1
  rc=$?; echo "tests v$v rc=$rc $(tail -n 1 $O/tests_v$v.log)"; [ $rc -ne 0 ] && exit $rc
done
for pass in 1 2; do for v in 0 1 2 3; do
  EXT_MPI_AMD_JOIN_CI_LOAD=$v timeout -k 10 240 python3 bench.py --shape joinci > $O/joinci_v${v}_$pass.json 2> $O/joinci_v$v.err || { tail -5 $O/joinci_v$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/joinci_v${v}_$pass.json').read())
print('joinci v$v pass $pass fused', d['fused']['avg_launch_us'], 'us | serial', d['serial']['avg_launch_us'])" | tee -a $O/summary.txt
done; done
port=29900
run() {  # N v pass
  port=$((port + 1))
  tag=n$1_v$2_$3
  EXT_MPI_AMD_JOIN_CI_LOAD=$2 timeout -k 10 150 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 --master-port $port bench.py --gpus $1 --steps 20 --warmup 5 \
    --child-transport node-ipc --child-result $O/${tag}_r{rank}.json --child-deadline 120 > $O/${tag}.log 2>&1 || { echo "$tag failed"; tail -5 $O/${tag}.log; return 1; }
  python3 -c "
import json; d=json.load(open('$O/${tag}_r0.json'))
print('$tag', 'start_to_wait %.1f' % (d['wall']*1e6/20), 'checked', d['checked'])" | tee -a $O/summary.txt
}
for pass in 1 2; do for N in 2 4; do for v in 0 1 2 3; do run $N $v $pass || exit 1; done; done; done
exit 0
