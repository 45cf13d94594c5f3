#!/bin/bash
# Round 5: the -k fractions through the leaf-major bucket map: parity (forced schedules), then the
# 16 MiB node launch of '6;-64 -8 8' under the per-tile and the leaf-major schedules beside the
# linear fold's leaf-major groups, two passes.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05/frac
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread \
  -k "leaf_major_chains or every_tuned" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for pass in 1 2; do
  for cp in "6;-64 -8 8" "6;1 -8 8"; do
    tag=$(echo "$cp" | tr -d ' ;-' )
    timeout -k 10 240 python bench.py --shape node16 --copyin "$cp" --schedules 524372,196626 > $O/${tag}_p$pass.json 2> $O/${tag}_p$pass.err || exit $?
    python3 -c "
import json; d=json.load(open('$O/${tag}_p$pass.json'))
print('$cp', 'pass $pass', ' '.join(f'{w}:{v[\"avg_launch_us\"]}{\"\" if v[\"checked\"] else \"!\"}' for w,v in d['by_schedule'].items()))"
  done
done
