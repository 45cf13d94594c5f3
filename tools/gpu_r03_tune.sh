#!/bin/bash
# Round-3: the multi-round schedule tuner (engine.c emac_tune) -- its parity test, then the bench.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "headline_instance or config2 or config3 or every_tuned" > gpurun_out/tune_tests.log 2>&1; rc=$?
tail -3 gpurun_out/tune_tests.log
[ $rc -ne 0 ] && exit $rc
EXT_MPI_AMD_DEBUG_TUNE=1 timeout -k 10 400 python -u bench.py > gpurun_out/tune_bench.json 2> gpurun_out/tune_bench.err; rc=$?
grep -c "schedule kept" gpurun_out/tune_bench.err
grep "schedule kept" gpurun_out/tune_bench.err | sort | uniq -c | sort -rn | head -20
exit $rc
