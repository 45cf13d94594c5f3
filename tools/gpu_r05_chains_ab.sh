#!/bin/bash
# Round 5: schedule words forced on the 16 MiB node launch for each fold tree (bench.py --shape node16
# --copyin ... --schedules), interleaved passes. Usage: gpu_r05_chains_ab.sh "<words>" <passes> <tag> [shape]
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05/${3:-ab}
mkdir -p $O
W="$1"; P=${2:-2}; SH=${4:-node16}
for pass in $(seq 1 $P); do
  for cp in "6;1 -8 8" "6;1 -2 -2 -2 2 2 2" "6;1 -4 -2 2 4" "6;1 -2 -4 4 2"; do
    tag=$(echo "$cp" | tr -d ' ;-' )
    timeout -k 10 240 python bench.py --shape $SH --copyin "$cp" --schedules $W > $O/${tag}_p$pass.json 2> $O/${tag}_p$pass.err || exit $?
    python3 -c "
import json,sys; d=json.load(open('$O/${tag}_p$pass.json'))
print('$cp', 'pass $pass', ' '.join(f'{w}:{v[\"avg_launch_us\"]}{\"\" if v[\"checked\"] else \"!\"}' for w,v in d['by_schedule'].items()))"
  done
done
