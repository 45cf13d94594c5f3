#!/bin/bash
# Round-3 PMC passes: memory-side request, DRAM credit-stall and UTCL1
# counters of the node fold (16 / 256 MiB per rank), the local fold (8 x 32 MiB -> 1), a 1:1 copy
# moving the node256 launch's bytes (the copy ceiling, same lease) and configs[2]'s int launch.
# One counter group per rocprofv3 run, no tracing domains; a pass that fails is reported and
# skipped, a pass killed by its time limit ends the script.
cd "$GRAFT_REPO_ROOT"
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # shape group counters...
  local shape=$1 group=$2; shift 2
  rm -rf gpurun_out/pmc3_${shape}_$group
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $R/gpurun_out/pmc3_${shape}_$group -o run --output-format csv -- \
    python3 $R/bench.py --shape $shape > gpurun_out/pmc3_${shape}_$group.json 2> gpurun_out/pmc3_${shape}_$group.err
  local rc=$?
  echo "pmc $shape $group rc=$rc"
  if [ $rc -eq 137 ] || [ $rc -eq 124 ]; then exit $rc; fi
  [ $rc -ne 0 ] && tail -n 3 gpurun_out/pmc3_${shape}_$group.err
  return 0
}
for shape in node256 copy256 local256 node16 int4; do
  run $shape ea TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum GRBM_GUI_ACTIVE
  run $shape stall TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum GRBM_GUI_ACTIVE
  run $shape tcp TCP_UTCL1_LFIFO_FULL_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE
done
python3 tools/pmc_counters.py gpurun_out/pmc3_node256_* gpurun_out/pmc3_local256_* gpurun_out/pmc3_node16_* gpurun_out/pmc3_int4_* > gpurun_out/pmc3_fold.json
python3 tools/pmc_counters.py --kernel=copy_k4 gpurun_out/pmc3_copy256_* > gpurun_out/pmc3_copy.json
cat gpurun_out/pmc3_fold.json gpurun_out/pmc3_copy.json
for s in node256 copy256 local256 node16 int4; do cat gpurun_out/pmc3_${s}_ea.json; done
exit 0
