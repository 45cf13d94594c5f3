#!/bin/bash
# Round-3: the driver's GPU suite and smoke(), then the node / local fold A/B harness.
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_r03_full.sh || exit $?
KIBS="2048 4096" bash tools/gpu_r03_nodevar.sh > gpurun_out/nodevar_all.txt 2>&1; rc=$?
grep -E "^node fold|burst|prod|local_u|copy|MISMATCH" gpurun_out/nodevar_all.txt
exit $rc
