#!/bin/bash
# Round 5: one load burst per leaf (fold_kernel.hpp kLeafBurst) -- the forced bitwise tests of every
# leaf-major form, then the 16 MiB node launch of the linear fold and the chains whose top level has
# radix 2 under the leaf-major forms, interleaved passes. Usage: gpu_r05_burst.sh <tag> <passes>
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05/${1:-burst}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "leaf_major_chains_forced" --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
W=196626,1245202,4390930  # leaf-major, its opening-copy form, one burst per leaf
for pass in $(seq 1 ${2:-2}); do
  for cp in "6;1 -8 8" "6;1 -2 -2 -2 2 2 2" "6;1 -4 -2 2 4" "6;1 -2 -4 4 2" "6;-64 -8 8"; do
    tag=$(echo "$cp" | tr -d ' ;-' )
    timeout -k 10 240 python bench.py --shape node16 --copyin "$cp" --schedules $W > $O/${tag}_p$pass.json 2> $O/${tag}_p$pass.err || exit $?
    python3 -c "
import json,sys; d=json.load(open('$O/${tag}_p$pass.json'))
print('$cp', 'pass $pass', ' '.join(f'{w}:{v[\"avg_launch_us\"]}{\"\" if v[\"checked\"] else \"!\"}' for w,v in d['by_schedule'].items()))" | tee -a $O/ab.txt
  done
done
# the 256 MiB point: its usual kept schedule (U 4 burst, buffer loads, device-scope stores) beside the leaf-major forms
timeout -k 10 300 python bench.py --shape node256 --schedules 786452,196626,4390930 > $O/node256.json 2> $O/node256.err || exit $?
python3 -c "
import json,sys; d=json.load(open('$O/node256.json'))
print('node256', ' '.join(f'{w}:{v[\"avg_launch_us\"]}{\"\" if v[\"checked\"] else \"!\"}' for w,v in d['by_schedule'].items()))" | tee -a $O/ab.txt
