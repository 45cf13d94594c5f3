#!/bin/bash
# Round-3: the multi-GPU bench path rehearsed on the one-GPU box after the peer-mapped node join
# (the N > 1 headline now runs with ranks sharing the GPU), and the 8-node join test.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 350 --timeout-method thread "tests/test_gpu_node_ipc.py::test_node_form_over_peer_mapped_nodes[8]" \
  > gpurun_out/nodeipc8.log 2>&1 || { tail -30 gpurun_out/nodeipc8.log; exit 1; }
tail -2 gpurun_out/nodeipc8.log
for n in 2 4; do
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --steps 20 --warmup 3 > gpurun_out/r03_bench_n$n.json 2> gpurun_out/r03_bench_n$n.err
  rc=$?
  echo "n=$n rc=$rc"
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/r03_bench_n$n.json').read().strip().splitlines()[-1])
print({k: d.get(k) for k in ('value','ms_per_step','n_gpus')}, d['config'].get('layout'), d['config'].get('transport'), d['config'].get('checked_vs_fp64_sum'))
print(d['roofline']); e=d['extras']; print(e.get('parts_us'), e.get('node_transports'))
" || tail -20 gpurun_out/r03_bench_n$n.err
  [ $rc -ne 0 ] && exit $rc
done
exit 0
