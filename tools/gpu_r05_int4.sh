#!/bin/bash
# Round 5: configs[2]'s int launch (4 MiB x 8, bench.py --shape int4) under leaf-major groups of 4
# vectors per lane (256 groups: one per CU) against the per-tile schedules, three passes; then the
# lease fingerprint. Usage: gpu_r05_int4.sh <lease tag>
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05/int4
mkdir -p $O
for pass in 1 2 3; do
  timeout -k 10 240 python bench.py --shape int4 --schedules 524372,20,163858,196625,688146 > $O/int4_p$pass.json 2> $O/int4_p$pass.err || exit $?
  python3 -c "
import json; d=json.load(open('$O/int4_p$pass.json'))
print('int4 pass $pass', ' '.join(f'{w}:{v[\"avg_launch_us\"]}{\"\" if v[\"checked\"] else \"!\"}' for w,v in d['by_schedule'].items()))"
done
bash tools/gpu_r05_lease.sh ${1:-int4}
