#!/bin/bash
# Round 6: the local fold (8 x 32 MiB -> 1) under each one-destination schedule
# forced (bench.py --shape local256 --schedules), two passes in opposite orders on one lease. W1 / W2
# (comma-separated schedule words, env) pick the schedules; TAG names the output directory. The
# first A/B also ran the LDS groups with buffer loads at 2 and 8 tiles: those kernels were slower
# and are no longer instantiated, so the default lists name the kept schedules
# (U 2, 4 tiles), (U 4, staggered, buffer loads), (U 4, 2 tiles), (U 4, burst) plus (U 4, 4
# tiles) and (U 2, burst), which the tuner now skips for this shape.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06/localab${TAG:+_$TAG}
mkdir -p $O
W1=${W1:-65554,524372,32788,20,65556,18}
W2=${W2:-18,65556,20,32788,524372,65554}
i=0
for w in $W1 $W2; do
  i=$((i + 1))
  timeout -k 10 400 python3 bench.py --shape local256 --schedules $w > $O/pass$i.json 2> $O/pass$i.err || { tail -5 $O/pass$i.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/pass$i.json').read())
for k, v in d['by_schedule'].items(): print('pass $i', k, v)" | tee -a $O/summary.txt
done
