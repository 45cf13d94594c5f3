#!/bin/bash
# Round 5: every fan-out schedule forced on the 256 MiB node launch, twice, then the lease
# fingerprint (is the best schedule of a slow lease another one?). Usage: gpu_r05_sched256.sh <tag>
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05/sched256/$1
mkdir -p $O
W=20,84,524372,786452,32788,65554,196626
for pass in 1 2; do
  timeout -k 10 400 python bench.py --shape node256 --schedules $W > $O/p$pass.json 2> $O/p$pass.err || exit $?
  python3 -c "
import json; d=json.load(open('$O/p$pass.json'))
print('node256 pass $pass', ' '.join(f'{w}:{v[\"avg_launch_us\"]}' for w,v in d['by_schedule'].items()))"
done
bash tools/gpu_r05_lease.sh $1
