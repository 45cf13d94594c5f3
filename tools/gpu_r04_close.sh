#!/bin/bash
# Round-4 closing call: the driver's GPU suite command, smoke(), the default bench, then the
# closing evidence (PMC traffic, the driver's bench command under rocprofv3 --stats).
cd "$GRAFT_REPO_ROOT"
tag=${1:-r04z}
bash tools/gpu_r04_check.sh $tag || exit $?
bash tools/gpu_r04_final.sh
