#!/bin/bash
# Round-3: DRAM credit stalls of the deferred-store schedule against the per-tile ones, same
# lease, same command (bench.py --shape: the handle's tuning runs every candidate 3 times, then the
# kept one). One counter group per rocprofv3 run, no tracing domains.
cd "$GRAFT_REPO_ROOT"
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # shape group counters...
  local shape=$1 group=$2; shift 2
  rm -rf gpurun_out/pmcd_${shape}_$group
  timeout -s KILL 150 rocprofv3 --pmc "$@" -d $R/gpurun_out/pmcd_${shape}_$group -o run --output-format csv -- \
    python3 $R/bench.py --shape $shape > gpurun_out/pmcd_${shape}_$group.json 2> gpurun_out/pmcd_${shape}_$group.err
  local rc=$?
  echo "pmc $shape $group rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 3 gpurun_out/pmcd_${shape}_$group.err; exit $rc; fi
}
for shape in node16 node256; do
  run $shape ea TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE
  run $shape stall TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum GRBM_GUI_ACTIVE
done
for shape in node16 node256; do
  for k in "8, 2, 0, 8, 4097>" "8, 4, 0, 8, 2049>" "8, 2, 0, 8, 6145>" "8, 2, 0, 8, 1>" "8, 4, 0, 8, 1>" "8, 4, 0, 8, 5>"; do
    echo "== $shape [$k]"
    python3 tools/pmc_counters.py "--kernel=$k" gpurun_out/pmcd_${shape}_ea gpurun_out/pmcd_${shape}_stall
  done
done > gpurun_out/pmcd_summary.txt
cat gpurun_out/pmcd_summary.txt | head -150
