#!/bin/bash
# Round 5: leaf-major groups over the compile-time radix chains. The forced-schedule parity tests,
# the tuner's every-candidate test, then each chain's schedules forced on the 16 MiB node launch
# (bench.py --shape node16 --copyin ... --schedules), two interleaved passes.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05
O=gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread \
  -k "leaf_major_chains or every_tuned" > $O/chains_tests.log 2>&1 || { tail -30 $O/chains_tests.log; exit 1; }
tail -3 $O/chains_tests.log
W="524372,196626,163858,65554,32788"
for pass in 1 2; do
  for cp in "6;1 -2 -2 -2 2 2 2" "6;1 -4 -2 2 4" "6;1 -2 -4 4 2"; do
    tag=$(echo "$cp" | tr -d ' ;-' )
    timeout -k 10 240 python bench.py --shape node16 --copyin "$cp" --schedules $W > $O/chain_${tag}_p$pass.json 2> $O/chain_${tag}_p$pass.err || exit $?
    echo "$cp pass $pass: $(cat $O/chain_${tag}_p$pass.json)"
  done
  timeout -k 10 240 python bench.py --shape node16 --schedules 196626,524372 > $O/linear_p$pass.json 2> $O/linear_p$pass.err || exit $?
  echo "linear pass $pass: $(cat $O/linear_p$pass.json)"
done
