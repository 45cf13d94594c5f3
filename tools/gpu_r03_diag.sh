#!/bin/bash
# Round-3 diagnosis: forced re-placement (EXT_MPI_AMD_IPC_FORCE_MIRROR=1) with 8 processes, the
# cases that failed in session A, with per-element mismatch reports.
cd "$GRAFT_REPO_ROOT"
export EXT_MPI_AMD_DEBUG_IPC=1 IPC_FUZZ=4
EXT_MPI_AMD_IPC_FORCE_MIRROR=1 IPC_CASES=7,22,7,0 IPC_SECTIONS=concurrent,newdata,recovery bash tools/gpu_ipc_worker.sh 8 forced8 || true
IPC_CASES=7,22,7,0 IPC_SECTIONS=concurrent,newdata bash tools/gpu_ipc_worker.sh 8 plain8 || true
EXT_MPI_AMD_IPC_FORCE_MIRROR=1 IPC_CASES=7,7,0,18 IPC_SECTIONS=concurrent,newdata,recovery bash tools/gpu_ipc_worker.sh 2 forced2 || true
grep -h "differ\|wrong\|refused\|unreachable\|cannot\|Error" gpurun_out/worker_forced8_r*.log | sort | uniq -c | sort -rn | head -40
