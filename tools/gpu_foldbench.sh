#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Iext_mpi_collectives_amd/csrc tools/foldbench.hip -o /tmp/foldbench -Lext_mpi_collectives_amd -lext_mpi_amd -Wl,-rpath,$PWD/ext_mpi_collectives_amd || exit 1
for mib in ${MIBS:-16 256}; do
  timeout -k 10 240 /tmp/foldbench $mib 7 20 > gpurun_out/foldbench_${mib}.txt 2>&1 || exit $?
  cat gpurun_out/foldbench_${mib}.txt
done
