#!/bin/bash
# Round-4 A/B: load issue order and spacing of (U 4) with buffer loads (ISSUE bit 0 source-major,
# bits 1.. s_sleep after every 4 loads), against the current candidates, two passes.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/spc4
mkdir -p $O
for rep in 1 2; do
  for shape in int4 node16 node64; do
    w="84,20,524372,524340,524436,524564,524356,524292,524404"
    timeout -k 10 300 python3 bench.py --shape $shape --schedules $w > $O/${shape}_$rep.json 2> $O/${shape}_$rep.err || { echo "$shape rc=$?"; tail -5 $O/${shape}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${shape}_$rep.json').read().strip().splitlines()[-1]); print('$rep $shape', {k: v['avg_launch_us'] for k, v in d['by_schedule'].items()})"
  done
done
exit 0
