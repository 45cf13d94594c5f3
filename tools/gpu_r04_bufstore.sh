#!/bin/bash
# Round-4 A/B: nontemporal buffer stores (kBufStore) and device-scope stores on the leaf-major
# groups, against the current candidates, each schedule forced in turn, two passes.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/bst4
mkdir -p $O
for rep in 1 2; do
  for shape in node16 node64 int4; do
    w="84,524372,1572948,1048660,196626,1245202,458770"
    timeout -k 10 300 python3 bench.py --shape $shape --schedules $w > $O/${shape}_$rep.json 2> $O/${shape}_$rep.err || { echo "$shape rc=$?"; tail -5 $O/${shape}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${shape}_$rep.json').read().strip().splitlines()[-1]); print('$rep $shape', {k: v['avg_launch_us'] for k, v in d['by_schedule'].items()})"
  done
done
exit 0
