#!/bin/bash
# Round 5: split leaf-major groups (fold_kernel.hpp kSplitTop) -- the forced bitwise tests of every
# leaf-major form, then the 16 MiB node launch of the linear fold and the chains whose top level has
# radix 2 under the unsplit and split forms, interleaved passes. Usage: gpu_r05_split.sh <tag> <passes>
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05/${1:-split}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "leaf_major_chains_forced" --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
W=196626,1245202,4358162,5406738  # leaf-major, its opening-copy form, split, split with opening copies
for pass in $(seq 1 ${2:-2}); do
  for cp in "6;1 -8 8" "6;1 -2 -2 -2 2 2 2" "6;1 -4 -2 2 4"; do
    tag=$(echo "$cp" | tr -d ' ;-' )
    timeout -k 10 240 python bench.py --shape node16 --copyin "$cp" --schedules $W > $O/${tag}_p$pass.json 2> $O/${tag}_p$pass.err || exit $?
    python3 -c "
import json,sys; d=json.load(open('$O/${tag}_p$pass.json'))
print('$cp', 'pass $pass', ' '.join(f'{w}:{v[\"avg_launch_us\"]}{\"\" if v[\"checked\"] else \"!\"}' for w,v in d['by_schedule'].items()))" | tee -a $O/ab.txt
  done
done
