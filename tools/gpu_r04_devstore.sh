#!/bin/bash
# Round-4 A/B: device-scope streaming stores (fold_kernel.hpp kDevStore) against the default
# nontemporal stores, each schedule forced in turn (bench.py --shape ... --schedules), two passes.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/dev4
mkdir -p $O
for rep in 1 2; do
  for shape in node16 node64 node256 int4; do
    w="84,262228,20,262164,196626,458770"
    timeout -k 10 300 python3 bench.py --shape $shape --schedules $w > $O/${shape}_$rep.json 2> $O/${shape}_$rep.err || { echo "$shape rc=$?"; tail -5 $O/${shape}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${shape}_$rep.json').read().strip().splitlines()[-1]); print('$rep $shape', {k: (v['avg_launch_us'], v['checked']) for k, v in d['by_schedule'].items()})"
  done
done
exit 0
