#!/bin/bash
# Round-4: the blocking MPI_Allreduce front end on device buffers over the default
# peer-mapped transport, staging through communicator scratch with two synchronous copies
# (EXT_MPI_AMD_SYNC_STAGE=1, round 3) or on the handle's stream (round 4), beside the persistent
# path on the same buffers; 2 and 4 MPI ranks sharing the one MI355X.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/blk4
mkdir -p $O
M=/opt/conda
L=ext_mpi_collectives_amd
gcc -O2 tools/mpi_blocking_time.c -o $O/mpi_blocking_time -Iinclude -I$M/include -L$L -lext_mpi_collectives -lext_mpi_amd \
  $M/lib/libmpi.so -Wl,-rpath-link,/lib/x86_64-linux-gnu -Wl,-rpath,$PWD/$L -Wl,-rpath,$M/lib || exit 1
for np in 2 4; do
  for n in 256 262144 4194304; do
    for sync in 1 0; do
      EXT_MPI_BLOCKING=1 EXT_MPI_AMD_ASYNC_STAGE=$((1-sync)) timeout -k 10 120 $M/bin/mpiexec -n $np $O/mpi_blocking_time $n 100 > $O/np${np}_n${n}_sync$sync.txt 2>&1
      rc=$?; echo "np=$np count=$n sync=$sync rc=$rc $(grep TIME $O/np${np}_n${n}_sync$sync.txt)"
      [ $rc -ne 0 ] && { tail -5 $O/np${np}_n${n}_sync$sync.txt; exit $rc; }
    done
  done
done
exit 0
