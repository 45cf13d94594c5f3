#!/bin/bash
# Round-4 A/B: leaf-major group shapes (U x KB vectors per lane per leaf) of the node fan-out,
# against the kept (U 2, 4 tiles), each forced in turn, two passes.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/lm4
mkdir -p $O
for rep in 1 2; do
  for shape in node16 node64 int4; do
    w="196626,229393,163860,163858,196628,229394,524372"
    timeout -k 10 300 python3 bench.py --shape $shape --schedules $w > $O/${shape}_$rep.json 2> $O/${shape}_$rep.err || { echo "$shape rc=$?"; tail -5 $O/${shape}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${shape}_$rep.json').read().strip().splitlines()[-1]); print('$rep $shape', {k: (v['avg_launch_us'], v['checked']) for k, v in d['by_schedule'].items()})"
  done
done
exit 0
