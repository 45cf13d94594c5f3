#!/bin/bash
# Round 6: the local fold (8 x 32 MiB -> 1) under each one-destination schedule
# forced (bench.py --shape local256 --schedules), two passes in opposite orders on one lease: the
# kept candidates (LDS groups U 2 / U 4 x 4 tiles, U 4 staggered with buffer loads) against the LDS
# groups with buffer loads, 2 and 8 tiles (fold_kernel.hpp, instantiated for this A/B).
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06/localab
mkdir -p $O
W1=65554,524372,65556,589842,589844,32788,98322
W2=98322,32788,589844,589842,65556,524372,65554
i=0
for w in $W1 $W2; do
  i=$((i + 1))
  timeout -k 10 400 python3 bench.py --shape local256 --schedules $w > $O/pass$i.json 2> $O/pass$i.err || { tail -5 $O/pass$i.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/pass$i.json').read())
for k, v in d['by_schedule'].items(): print('pass $i', k, v)" | tee -a $O/summary.txt
done
