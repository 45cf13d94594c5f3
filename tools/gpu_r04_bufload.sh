#!/bin/bash
# Round-4 A/B: leaf loads as buffer loads (fold_kernel.hpp kBufLoad) against global loads, each
# schedule forced in turn (bench.py --shape ... --schedules), pairs adjacent, two passes.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/buf4
mkdir -p $O
for rep in 1 2; do
  for shape in node16 node256 int4 local256; do
    if [ $shape = local256 ]; then w="20,524308,65554,589842,65556,589844"; else w="84,524372,20,524308,262164,786452,196626,720914"; fi
    timeout -k 10 300 python3 bench.py --shape $shape --schedules $w > $O/${shape}_$rep.json 2> $O/${shape}_$rep.err || { echo "$shape rc=$?"; tail -5 $O/${shape}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${shape}_$rep.json').read().strip().splitlines()[-1]); print('$rep $shape', {k: v['avg_launch_us'] for k, v in d['by_schedule'].items()})"
  done
done
exit 0
