#!/bin/bash
# HBM traffic of the bench's fold launch from rocprofv3 PMC counters: FETCH_SIZE and WRITE_SIZE in
# separate passes (each its own run, no tracing domains), then tools/pmc_traffic.py applies the
# gfx950 corrections and writes profiles/traffic_<tag>.json.
set -u
cd "$GRAFT_REPO_ROOT"
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/pmc_$c
  timeout -s KILL 120 rocprofv3 --pmc $c -d $R/gpurun_out/pmc_$c -o run --output-format csv -- \
    python3 $R/bench.py --no-extras --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/pmc_$c.json 2> gpurun_out/pmc_$c.err
  rc=$?
  echo "pmc $c rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_$c.err; exit $rc; fi
done
python3 tools/pmc_traffic.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE gpurun_out/traffic.json node_r8_16mib_float
