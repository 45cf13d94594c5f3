#!/bin/bash
# Round-2 PMC passes (rocprofv3 --pmc, one counter group per run, no tracing domains): HBM bytes of
# the local fold (8 x 32 MiB -> 1) and the node-form fold at 256 MiB per rank, and translation /
# Infinity-Cache counters for the 256 MiB node launch. Writes gpurun_out/pmc_r02_<shape>_<ctr>/.
set -u
cd "$GRAFT_REPO_ROOT"
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # shape counters...
  local shape=$1; shift
  local tag=$(echo "$*" | tr ' ' '_')
  rm -rf gpurun_out/pmc_r02_${shape}_$tag
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d $R/gpurun_out/pmc_r02_${shape}_$tag -o run --output-format csv -- \
    python3 $R/bench.py --shape $shape > gpurun_out/pmc_r02_${shape}_$tag.json 2> gpurun_out/pmc_r02_${shape}_$tag.err
  local rc=$?
  echo "pmc $shape $* rc=$rc"
  [ $rc -ne 0 ] && { tail -n 5 gpurun_out/pmc_r02_${shape}_$tag.err; exit $rc; }
  return 0
}
timeout -k 5 60 rocprofv3 --list-avail > gpurun_out/pmc_list_avail.txt 2>&1
for shape in local256 node256 node16; do
  run $shape FETCH_SIZE
  run $shape WRITE_SIZE
done
exit 0
