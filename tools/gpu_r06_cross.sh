#!/bin/bash
# Round 6, VERDICT r05 items 1-2 (one gpurun call):
#  1. the cross-GPU code on one GPU (EXT_MPI_AMD_TEST_CROSS_DEVICE=1) under the bitwise node-IPC
#     and peer-mapped tests, plus the join settings agreed on rank 0;
#  2. a kernel + HIP runtime trace of two node-IPC workers with and without the hook: the
#     join_fused_kernel<..., true> instantiation and the extra release records (hipEventRecord);
#  3. the fused join's copy-in alone (bench.py --shape joinci) timed, then PMC passes of it:
#     FETCH_SIZE / WRITE_SIZE (traffic) and the DRAM credit stalls / in-flight levels.
cd "$GRAFT_REPO_ROOT"
R=$PWD
O=gpurun_out/r06/cross
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_node_ipc.py tests/test_gpu_peer_mapped.py -k "cross_device or follow_rank0" > $O/tests.log 2>&1
rc=$?
tail -n 25 $O/tests.log
[ $rc -ne 0 ] && exit $rc
trace() {  # tag, extra env: two node_ipc_worker processes, each under its own rocprofv3
  local tag=$1; shift
  local port=$((29700 + RANDOM % 200)) pids=()
  for r in 0 1; do
    env RANK=$r WORLD_SIZE=2 LOCAL_RANK=$r MASTER_ADDR=127.0.0.1 MASTER_PORT=$port IPC_DEVICE=0 \
      EXT_MPI_AMD_BARRIER_TIMEOUT=20 "$@" \
      timeout -k 10 240 rocprofv3 --kernel-trace --hip-runtime-trace --stats -d $R/$O/trace_$tag/r$r -o run \
      --output-format csv -- python3 $R/tests/node_ipc_worker.py > $O/trace_${tag}_r$r.log 2>&1 &
    pids+=($!)
  done
  local bad=0
  for p in "${pids[@]}"; do wait $p || bad=1; done
  echo "trace $tag: $(grep -c ': ok' $O/trace_${tag}_r0.log) ok lines, rc bad=$bad"
  return $bad
}
trace cross EXT_MPI_AMD_TEST_CROSS_DEVICE=1 || exit 1
trace same EXT_MPI_AMD_TEST_CROSS_DEVICE=0 || exit 1
python3 - $O <<'PY'
import csv, glob, sys
o = sys.argv[1]
for tag in ("cross", "same"):
    ks, api = {}, {}
    for f in glob.glob(f"{o}/trace_{tag}/**/*kernel_stats.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if "join_fused" in row["Name"]:
                ks[row["Name"][:90]] = ks.get(row["Name"][:90], 0) + int(row["Calls"])
    for f in glob.glob(f"{o}/trace_{tag}/**/*hip_api_stats.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Name"] in ("hipEventRecord", "hipEventRecordWithFlags", "hipLaunchKernel", "hipExtLaunchKernel"):
                api[row["Name"]] = api.get(row["Name"], 0) + int(row["Calls"])
    print(tag, "join_fused_kernel instances:", ks, "| api calls:", api)
PY
find $O/trace_cross $O/trace_same -name "*_trace.csv" -size +4M -delete  # the stats files stay
# the fused copy-in alone, then under PMC (every join_fused_kernel dispatch is a copy-in)
for g in 0 512; do
  if [ $g = 0 ]; then unset EXT_MPI_AMD_JOIN_GRID; else export EXT_MPI_AMD_JOIN_GRID=$g; fi
  timeout -k 10 240 python3 bench.py --shape joinci > $O/joinci_g$g.json 2> $O/joinci_g$g.err || { tail -5 $O/joinci_g$g.err; exit 1; }
  echo "joinci grid $g: $(cat $O/joinci_g$g.json)"
done
unset EXT_MPI_AMD_JOIN_GRID
pass() {  # group counters...
  local group=$1; shift
  rm -rf $O/pmc_joinci_$group
  timeout -s KILL 180 rocprofv3 --pmc "$@" -d $R/$O/pmc_joinci_$group -o run --output-format csv -- \
    python3 $R/bench.py --shape joinci > $O/pmc_joinci_$group.json 2> $O/pmc_joinci_$group.err
  local rc=$?
  echo "pmc joinci $group rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 3 $O/pmc_joinci_$group.err; exit $rc; fi
}
pass FETCH_SIZE FETCH_SIZE
pass WRITE_SIZE WRITE_SIZE
pass stall TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum GRBM_GUI_ACTIVE
pass level TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE
python3 tools/pmc_traffic.py $O/pmc_joinci_FETCH_SIZE $O/pmc_joinci_WRITE_SIZE $O/traffic_joinci_fused.json joinci_fused 'join_fused_kernel<'
python3 tools/pmc_traffic.py $O/pmc_joinci_FETCH_SIZE $O/pmc_joinci_WRITE_SIZE $O/traffic_joinci_serial.json joinci_serial
python3 tools/pmc_counters.py --by-kernel '--kernel=join_fused_kernel|fold_' $O/pmc_joinci_* > $O/pmc_joinci.json
cat $O/traffic_joinci_*.json
for f in $(find $O -name "*counter_collection*.csv"); do  # keep the join's and the folds' rows only
  python3 -c "
import sys
rows = open(sys.argv[1]).read().splitlines()
open(sys.argv[1], 'w').write('\n'.join(rows[:1] + [r for r in rows[1:] if 'fold_' in r or 'join_fused' in r]) + '\n')" $f
done
exit 0
