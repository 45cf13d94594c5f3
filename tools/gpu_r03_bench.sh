#!/bin/bash
# Round-3: the default N = 1 bench (tuner debug on), its JSON line summarised.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
EXT_MPI_AMD_DEBUG_TUNE=1 timeout -k 10 500 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
[ $rc -ne 0 ] && { tail -20 gpurun_out/bench.err; exit $rc; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/bench.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["config"]["fold_schedule"])
print(d["roofline"])
e = d["extras"]
for k in ("read_variants_gbps", "write_variants_gbps", "copy_variants_gbps", "point_256MiB", "local_fold_256MiB", "config3_int_long_4MiB"):
    print(k, e.get(k))
print(d["cpu_baseline"]["value"], d["cpu_baseline"]["cores"])
PY
