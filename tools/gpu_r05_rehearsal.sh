#!/bin/bash
# Round 5: the N > 1 bench rehearsed with N processes sharing the one MI355X, the fused pipelined
# join as the default (engine_join.c), bounded as the driver's run would be. Usage: gpu_r05_rehearsal.sh N...
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05/rehearsal
mkdir -p $O
for n in "$@"; do
  EXT_MPI_AMD_BENCH_DEADLINE=420 timeout -k 10 560 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29620 + n)) bench.py --gpus $n --steps 10 --warmup 3 \
    > $O/bench_n${n}.json 2> $O/bench_n${n}.err
  rc=$?
  echo "rehearsal n=$n rc=$rc"
  [ $rc -ne 0 ] && { tail -20 $O/bench_n${n}.err; exit $rc; }
  python3 - $O/bench_n${n}.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e = d.get('extras', {})
print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'transport', d['config'].get('transport'), 'join_parts', e.get('join_parts'))
print('parts_us', e.get('parts_us'))
print('failures', [(f.get('transport'), f.get('rank'), f.get('exit')) for f in e.get('failures', [])])
PY
done
