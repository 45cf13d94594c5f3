#!/bin/bash
# Round-3: the staggered fan-out schedule's s_sleep (ISSUE bits 1-7) forced on the bench's shapes:
# 84 = (U 4, s_sleep 2 every 4 loads), 52 = s_sleep 1, 148 = s_sleep 4, 20 = burst. (52 and 148
# were instantiated for this run only: profiles/r03_tune/sleep_ab.txt)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/sleep_ab.txt
one() {  # rep schedule bench-args...
  local rep=$1 s=$2; shift 2
  EXT_MPI_AMD_FOLD_SCHEDULE=$s timeout -k 10 200 python3 -u bench.py "$@" > gpurun_out/fab.json 2> gpurun_out/fab.err || { tail -5 gpurun_out/fab.err; exit 1; }
  python3 - "$s" "$rep" >> gpurun_out/sleep_ab.txt <<'PY'
import json, sys
d = json.loads(open("gpurun_out/fab.json").read().strip().splitlines()[-1])
if "roofline" in d:
    print(sys.argv[2], sys.argv[1], "headline", d["roofline"]["avg_launch_us"], d["config"]["fold_schedule"], d["config"]["checked_vs_fp64_sum"])
else:
    print(sys.argv[2], sys.argv[1], d["shape"], d["avg_launch_us"], d["schedule"], d["checked"])
PY
  tail -1 gpurun_out/sleep_ab.txt
}
for rep in 1 2; do
  for s in 84 52 148 20; do one $rep $s --no-extras --no-cpu-baseline --steps 50; done
  for s in 84 52 148 20; do one $rep $s --shape node256; done
  for s in 84 52 148 20; do one $rep $s --shape int4; done
done
