#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 tools/pipebench 32 7 10 > gpurun_out/pipe32.txt 2>&1; echo rc=$?
cat gpurun_out/pipe32.txt
timeout -k 10 200 tools/pipebench 4 7 20 > gpurun_out/pipe4.txt 2>&1; echo rc=$?
cat gpurun_out/pipe4.txt
