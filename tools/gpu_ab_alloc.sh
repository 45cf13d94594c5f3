#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for a in hip torch hip torch; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --alloc $a > gpurun_out/ab_$a.json 2> gpurun_out/ab_$a.err || exit $?
  python -c "
import json; d=json.load(open('gpurun_out/ab_$a.json')); print('$a', d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['extras']['point_256MiB'])"
done
