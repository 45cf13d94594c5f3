#!/bin/bash
# Round-3: the tuner's candidates at small launches (U 1 in place of the 8-tile deferred schedule
# under 8 MiB per leaf): the tuned-schedule parity test, then the bench with the tuner's debug lines.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "every_tuned_schedule or tuned_fold" --timeout 120 --timeout-method thread > gpurun_out/small_tests.log 2>&1 || { tail -30 gpurun_out/small_tests.log; exit 1; }
tail -2 gpurun_out/small_tests.log
EXT_MPI_AMD_DEBUG_TUNE=1 timeout -k 10 500 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
grep "kept" gpurun_out/bench.err
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/bench.json").read().strip().splitlines()[-1])
print(d["value"], d["roofline"]["avg_launch_us"], d["roofline"]["frac"], d["config"]["fold_schedule"])
print(d["extras"].get("config3_int_long_4MiB"))
PY
