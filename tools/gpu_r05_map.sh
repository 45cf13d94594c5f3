#!/bin/bash
# Round 5: the `-k` fractions' bucket map held in each wave's registers (fold_kernel.hpp deferred_body
# MAP: no LDS table, no barrier) -- the whole GPU suite, then the 16 MiB node launch of the linear
# fold and the `-64` fractions under the leaf-major forms, interleaved passes. Usage: gpu_r05_map.sh <tag> <passes>
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05/${1:-map}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
W=196626,1245202  # leaf-major, its opening-copy form
for pass in $(seq 1 ${2:-3}); do
  for cp in "6;1 -8 8" "6;-64 -8 8" "6;-64 -2 -2 -2 2 2 2"; do
    tag=$(echo "$cp" | tr -d ' ;-' )
    timeout -k 10 240 python bench.py --shape node16 --copyin "$cp" --schedules $W > $O/${tag}_p$pass.json 2> $O/${tag}_p$pass.err || exit $?
    python3 -c "
import json,sys; d=json.load(open('$O/${tag}_p$pass.json'))
print('$cp', 'pass $pass', ' '.join(f'{w}:{v[\"avg_launch_us\"]}{\"\" if v[\"checked\"] else \"!\"}' for w,v in d['by_schedule'].items()))" | tee -a $O/ab.txt
  done
done
