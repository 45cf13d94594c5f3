#!/bin/bash
# Round-3: the tuner's per-candidate times on single shapes (bench.py --shape), EXT_MPI_AMD_DEBUG_TUNE=1.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for sh in ${SHAPES:-local256 node16 node256}; do
  EXT_MPI_AMD_DEBUG_TUNE=1 timeout -k 10 200 python -u bench.py --shape $sh > gpurun_out/shape_$sh.json 2> gpurun_out/shape_$sh.err || exit $?
  echo "== $sh: $(cat gpurun_out/shape_$sh.json)"
  grep "schedule kept" gpurun_out/shape_$sh.err | head -12
done
