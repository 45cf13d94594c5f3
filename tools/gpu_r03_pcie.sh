#!/bin/bash
# Round-3: PCIe legs of the host-buffer path (tools/pcieprobe.hip).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 tools/pcieprobe 128 5 > gpurun_out/pcieprobe_128.txt 2>&1; rc=$?
cat gpurun_out/pcieprobe_128.txt
exit $rc
