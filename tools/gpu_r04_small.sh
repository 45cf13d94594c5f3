#!/bin/bash
# Round-4, BASELINE configs[2]'s launch size class: the int node form at 0.5 -
# 16 MiB per rank against a copy of the same bytes (bench.py --shape small: fixed cost and
# streaming rate from a line fit), the same sweep under the kernel tracer (per-dispatch durations
# and the gaps between dispatches), and every fan-out schedule at 4 MiB per rank.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/small4
mkdir -p $O
timeout -k 10 300 python3 bench.py --shape small > $O/sweep.json 2> $O/sweep.err || { echo "sweep rc=$?"; tail -5 $O/sweep.err; exit 1; }
cat $O/sweep.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 bench.py --shape small > $O/sweep_traced.json 2> $O/sweep_traced.err || { echo "traced rc=$?"; tail -5 $O/sweep_traced.err; exit 1; }
cat $O/sweep_traced.json
timeout -k 10 300 python3 bench.py --shape int4 --schedules 17,18,20,84,65554,32788,98322,196626 > $O/int4_sched.json 2> $O/int4_sched.err || { echo "sched rc=$?"; tail -5 $O/int4_sched.err; exit 1; }
cat $O/int4_sched.json
exit 0
