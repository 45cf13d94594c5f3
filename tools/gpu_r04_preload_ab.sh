#!/bin/bash
# Round-4 A/B: kernel arguments preloaded into SGPRs (-mllvm -amdgpu-kernarg-preload-count=16, the
# in-tree build) against the same sources without (tools/ab/libext_mpi_amd.so, KARG_PRELOAD=0),
# interleaved twice, on configs[2]'s int launch (4 MiB x 8), the 16 MiB headline fold and 256 MiB.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab4
mkdir -p $O
for rep in 1 2; do
  for shape in int4 node16 node256; do
    for v in pre nopre; do
      if [ $v = nopre ]; then export EXT_MPI_AMD_LIB=$PWD/tools/ab/libext_mpi_amd.so; else unset EXT_MPI_AMD_LIB; fi
      timeout -k 10 240 python3 bench.py --shape $shape > $O/${shape}_${v}_$rep.json 2> $O/${shape}_${v}_$rep.err || { echo "$shape $v rc=$?"; tail -3 $O/${shape}_${v}_$rep.err; exit 1; }
      echo "$rep $shape $v $(cat $O/${shape}_${v}_$rep.json)"
    done
  done
done
unset EXT_MPI_AMD_LIB
for k in 0 1; do
  HIP_FORCE_DEV_KERNARG=$k timeout -k 10 240 python3 bench.py --shape int4 > $O/int4_kernarg$k.json 2>/dev/null && echo "HIP_FORCE_DEV_KERNARG=$k $(cat $O/int4_kernarg$k.json)"
done
exit 0
