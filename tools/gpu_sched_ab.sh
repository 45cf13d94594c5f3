#!/bin/bash
# Launch-schedule A/B on this lease: node-form fold at 2 / 4 / 16 / 64 / 256 MiB per rank and the
# local fold at 4 / 32 MiB per leaf, interleaved rounds per size. Usage: bash tools/gpu_sched_ab.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
out=gpurun_out/sched_ab_$1.txt
: > $out
for m in 2 4 16 64 256; do timeout -k 10 120 ./tools/nodebench $m 9 $([ $m -ge 64 ] && echo 4 || echo 10) >> $out 2>&1 || exit 1; done
for m in 4 32; do timeout -k 10 120 ./tools/localbench $m 9 10 >> $out 2>&1 || exit 1; done
cat $out
