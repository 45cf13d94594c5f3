#!/bin/bash
# Round-3: fold schedules forced (EXT_MPI_AMD_FOLD_SCHEDULE, one candidate) against the tuner's
# own pick, interleaved on one lease, steady-state time per launch: the headline bench (16 MiB
# per rank), and the node256 / int4 shapes. 65554 = (U 2, 4 tiles, LDS groups), 196626 = its
# leaf-major form, 84 = (U 4, staggered), 20 = (U 4, burst).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/force_ab.txt
one() {  # rep schedule bench-args...
  local rep=$1 s=$2; shift 2
  if [ $s = tuner ]; then env_s=""; else env_s="EXT_MPI_AMD_FOLD_SCHEDULE=$s"; fi
  env $env_s timeout -k 10 200 python3 -u bench.py "$@" > gpurun_out/fab.json 2> gpurun_out/fab.err || { tail -5 gpurun_out/fab.err; exit 1; }
  python3 - "$s" "$rep" "$*" >> gpurun_out/force_ab.txt <<'PY'
import json, sys
d = json.loads(open("gpurun_out/fab.json").read().strip().splitlines()[-1])
if "roofline" in d:
    print(sys.argv[2], sys.argv[1], "headline", d["roofline"]["avg_launch_us"], d["config"]["fold_schedule"], d["config"]["checked_vs_fp64_sum"])
else:
    print(sys.argv[2], sys.argv[1], d["shape"], d["avg_launch_us"], d["schedule"], d["checked"])
PY
  tail -1 gpurun_out/force_ab.txt
}
for rep in 1 2; do
  for s in tuner 65554 196626; do one $rep $s --no-extras --no-cpu-baseline --steps 50; done
  for s in tuner 65554 196626 84 20; do one $rep $s --shape node256; done
  for s in tuner 65554 196626 84 20; do one $rep $s --shape int4; done
done
