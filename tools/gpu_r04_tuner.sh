#!/bin/bash
# Round-4: the tuner tests alone, then the default bench.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
tag=${1:-r04}
timeout -k 10 600 python -u -m pytest tests/test_gpu_tuner.py tests/test_gpu_parity.py -x -v -s -m gpu -k "tune or tuned or copy_reduce_headline" --timeout 300 --timeout-method thread > gpurun_out/${tag}_tuner_tests.log 2>&1
rc=$?
tail -25 gpurun_out/${tag}_tuner_tests.log
[ $rc -ne 0 ] && { echo "TUNER TESTS rc=$rc"; exit $rc; }
EXT_MPI_AMD_DEBUG_TUNE=1 timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || exit $?
grep "fold schedule kept" gpurun_out/${tag}_bench.err | head -20
tail -c 1500 gpurun_out/${tag}_bench.json
