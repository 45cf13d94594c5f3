#!/bin/bash
# Round 5: leaf-major groups for the one-destination local fold (8 x 32 MiB -> 1, bench.py --shape
# local256) against its kept schedules, and the -k fractions' node launch, two passes.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05/local
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread \
  -k "leaf_major_chains or every_tuned" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for pass in 1 2; do
  timeout -k 10 300 python bench.py --shape local256 --schedules 524372,65554,65556,196626,196628,229394,720916 > $O/local_p$pass.json 2> $O/local_p$pass.err || exit $?
  python3 -c "
import json; d=json.load(open('$O/local_p$pass.json'))
print('local256 pass $pass', ' '.join(f'{w}:{v[\"avg_launch_us\"]}' for w,v in d['by_schedule'].items()))"
  for cp in "6;-64 -8 8" "6;1 -8 8"; do
    tag=$(echo "$cp" | tr -d ' ;-' )
    timeout -k 10 240 python bench.py --shape node16 --copyin "$cp" --schedules 524372,196626 > $O/${tag}_p$pass.json 2> $O/${tag}_p$pass.err || exit $?
    python3 -c "
import json; d=json.load(open('$O/${tag}_p$pass.json'))
print('$cp', 'pass $pass', ' '.join(f'{w}:{v[\"avg_launch_us\"]}{\"\" if v[\"checked\"] else \"!\"}' for w,v in d['by_schedule'].items()))"
  done
done
