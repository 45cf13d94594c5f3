#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel trace. Stops at the first
# GPU fault / abort / timeout (exit codes other than 0 and pytest's 1).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 600 python -m pytest tests -m gpu -q ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -15 gpurun_out/gpu_tests.log
if fatal $rc; then exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 420 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
if [ $rc -ne 0 ]; then exit $rc; fi
if [ -n "${PROFILE:-1}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-extras > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err; rc=$?
  echo "rocprof rc=$rc"; tail -3 gpurun_out/bench_prof.err
  find gpurun_out/prof -name "*stats*" | head
fi
exit 0
