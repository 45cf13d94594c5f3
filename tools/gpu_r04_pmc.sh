#!/bin/bash
# Round-4: the node-form fold at 16 / 64 / 256 / 512 MiB per rank and the
# 1:1 copies of the 256 MiB launch's 4 GiB, on one lease: event timing of every fan-out schedule
# (EXT_MPI_AMD_FOLD_SCHEDULE), then rocprofv3 PMC passes, one counter group per run and no tracing
# domain: memory-side requests, DRAM credit stalls, in-flight levels, UTCL1 / UTCL2 translation.
# A pass that fails is reported and skipped; one killed by its time limit ends the script.
cd "$GRAFT_REPO_ROOT"
R=$PWD
O=gpurun_out/pmc4
mkdir -p $O
export TMPDIR=/tmp
ALL="20,84,32788,65554,196626"   # U4 burst, U4 staggered, (U4, 2 tiles), (U2, 4 tiles), leaf-major (U2, 4 tiles)
TWO="20,32788"
for sz in 16 64 256 512; do
  timeout -k 10 300 python3 bench.py --shape node$sz --schedules $ALL > $O/time_node$sz.json 2> $O/time_node$sz.err
  rc=$?; echo "time node$sz rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/time_node$sz.err; exit $rc; }
  cat $O/time_node$sz.json
done
# configs[2]'s int launch: U4 burst, U4 staggered, U2 burst, U2 / U1 half grid (two tiles per workgroup), U1 burst
timeout -k 10 300 python3 bench.py --shape int4 --schedules 20,84,18,262162,262161,17 > $O/time_int4.json 2> $O/time_int4.err
echo "time int4 rc=$? $(cat $O/time_int4.json)"
timeout -k 10 300 python3 bench.py --shape copy256 > $O/time_copy256.json 2> $O/time_copy256.err || exit $?
cat $O/time_copy256.json
# address translation A/B: the same launches on physically contiguous memory (hipDeviceMallocContiguous)
timeout -k 10 300 python3 bench.py --shape node256 --alloc contig --schedules $TWO > $O/time_node256_contig.json 2> $O/time_node256_contig.err
echo "time node256 contig rc=$? $(cat $O/time_node256_contig.json)"
timeout -k 10 300 python3 bench.py --shape copy256 --alloc contig > $O/time_copy256_contig.json 2> $O/time_copy256_contig.err
echo "time copy256 contig rc=$? $(cat $O/time_copy256_contig.json)"
pass() {  # shape group counters...
  local shape=$1 group=$2; shift 2
  local extra=""
  [ "${shape#node}" != "$shape" ] && extra="--schedules $TWO"
  [ "$group" = tlbcontig ] && extra="$extra --alloc contig"
  rm -rf $O/${shape}_$group
  timeout -s KILL 240 rocprofv3 --pmc "$@" -d $R/$O/${shape}_$group -o run --output-format csv -- \
    python3 $R/bench.py --shape $shape $extra > $O/${shape}_$group.json 2> $O/${shape}_$group.err
  local rc=$?
  echo "pmc $shape $group rc=$rc"
  if [ $rc -eq 137 ] || [ $rc -eq 124 ]; then exit $rc; fi
  [ $rc -ne 0 ] && tail -n 3 $O/${shape}_$group.err
  return 0
}
for shape in node16 node64 node256 node512 copy256; do
  pass $shape ea TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum GRBM_GUI_ACTIVE
  pass $shape stall TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum GRBM_GUI_ACTIVE
  pass $shape level TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_LEVEL_sum GRBM_GUI_ACTIVE
  pass $shape tlb TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_LFIFO_FULL_sum GRBM_GUI_ACTIVE
  pass $shape utcl2 GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE
done
pass node256 tlbcontig TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_LFIFO_FULL_sum GRBM_GUI_ACTIVE
python3 tools/pmc_counters.py --by-kernel $O/node16_* $O/node64_* $O/node256_* $O/node512_* > $O/pmc_fold.json
python3 tools/pmc_counters.py --by-kernel --kernel='copy_k4|copy_phased' $O/copy256_* > $O/pmc_copy.json
python3 tools/pmc_r04_summary.py $O > $O/summary.json
find $O -name "*counter_collection*.csv" -size +2M -delete  # keep what merges back small
ls -la $O | head -60
exit 0
