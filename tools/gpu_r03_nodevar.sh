#!/bin/bash
# Round-3: node-fold / local-fold variant A/B (tools/nodevar.hip) at configs[1]'s 16 MiB per rank,
# 32 MiB per rank (the local fold 8 x 32 MiB -> 1 of bench.py) and 256 MiB per rank.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for kib in ${KIBS:-2048 4096 32768}; do
  r=7; p=10; [ $kib -gt 4096 ] && { r=5; p=4; }
  timeout -k 10 300 tools/nodevar $kib $r $p > gpurun_out/nodevar_$kib.txt 2>&1 || exit $?
  cat gpurun_out/nodevar_$kib.txt
done
