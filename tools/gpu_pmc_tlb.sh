#!/bin/bash
# Translation and memory-side request counters of the node-form fold at 16 and 256 MiB per rank
# (does the 256 MiB launch lose time to address translation?). One counter group per run, no
# tracing domains. Writes gpurun_out/pmc_tlb_<shape>_<group>/ and gpurun_out/pmc_tlb.json.
set -u
cd "$GRAFT_REPO_ROOT"
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # shape group counters...
  local shape=$1 group=$2; shift 2
  rm -rf gpurun_out/pmc_tlb_${shape}_$group
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d $R/gpurun_out/pmc_tlb_${shape}_$group -o run --output-format csv -- \
    python3 $R/bench.py --shape $shape > gpurun_out/pmc_tlb_${shape}_$group.json 2> gpurun_out/pmc_tlb_${shape}_$group.err
  local rc=$?
  echo "pmc $shape $group rc=$rc"
  [ $rc -ne 0 ] && { tail -n 5 gpurun_out/pmc_tlb_${shape}_$group.err; exit $rc; }
  return 0
}
for shape in node16 node256; do
  run $shape utcl1 TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum
  run $shape utcl1b TCP_UTCL1_PERMISSION_MISS_sum TCP_UTCL1_SERIALIZATION_STALL_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum TCP_UTCL1_LFIFO_FULL_sum
  run $shape ea TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_WRITE_DRAM_sum
  run $shape stall TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum GRBM_GUI_ACTIVE
done
python3 tools/pmc_counters.py gpurun_out/pmc_tlb_* > gpurun_out/pmc_tlb.json
cat gpurun_out/pmc_tlb.json
exit 0
