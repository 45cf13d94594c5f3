#!/bin/bash
# Round-4 check: the driver's GPU suite command, smoke(), then the default bench (N = 1).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
tag=${1:-r04}
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread --durations=15 > gpurun_out/${tag}_gpu_tests.log 2>&1
rc=$?
tail -25 gpurun_out/${tag}_gpu_tests.log
[ $rc -ne 0 ] && { echo "GPU SUITE rc=$rc"; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${tag}_smoke.log 2>&1 || exit $?
tail -2 gpurun_out/${tag}_smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || exit $?
tail -c 600 gpurun_out/${tag}_bench.json
