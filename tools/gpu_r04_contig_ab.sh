#!/bin/bash
# Round-4 A/B of address translation: the node fold on hipMalloc buffers against physically
# contiguous ones (hipExtMallocWithFlags hipDeviceMallocContiguous, bench.py --alloc contig),
# default (tuned) schedule, interleaved twice; then the UTCL2 busy share of the contiguous runs.
cd "$GRAFT_REPO_ROOT"; R=$PWD
O=gpurun_out/contig4
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for shape in node16 node64 node256 int4; do
    for a in hip contig; do
      timeout -k 10 240 python3 bench.py --shape $shape --alloc $a > $O/${shape}_${a}_$rep.json 2> $O/${shape}_${a}_$rep.err || { echo "$shape $a rc=$?"; tail -3 $O/${shape}_${a}_$rep.err; exit 1; }
      echo "$rep $shape $a $(cat $O/${shape}_${a}_$rep.json)"
    done
  done
done
for shape in node16 node256; do
  for a in hip contig; do
    rm -rf $O/pmc_${shape}_$a
    timeout -s KILL 240 rocprofv3 --pmc GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE -d $R/$O/pmc_${shape}_$a -o run --output-format csv -- \
      python3 $R/bench.py --shape $shape --alloc $a > $O/pmc_${shape}_$a.json 2> $O/pmc_${shape}_$a.err
    rc=$?; echo "pmc $shape $a rc=$rc"; [ $rc -eq 137 ] && exit $rc
  done
done
python3 tools/pmc_counters.py --by-kernel $O/pmc_* > $O/utcl2.json
cat $O/utcl2.json | head -60
exit 0
