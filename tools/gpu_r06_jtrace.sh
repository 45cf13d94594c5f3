#!/bin/bash
# Round 6: where the fused node join's time goes -- per-workgroup timelines (EXT_MPI_AMD_JOIN_TRACE,
# join_fused.hip) of the copy-ins alone (bench.py --shape joinci, mode 1) and of whole Starts at N = 1
# and N = 2 (processes sharing the GPU), summarised by tools/join_trace_summary.py. The joinci shape
# is timed without the trace first (the trace synchronises between launches).
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06/jtrace
mkdir -p $O
rm -f $O/*.trace.*
timeout -k 10 240 python3 bench.py --shape joinci > $O/joinci_notrace.json 2> $O/joinci_notrace.err || { tail -5 $O/joinci_notrace.err; exit 1; }
echo "joinci (no trace): $(cat $O/joinci_notrace.json)"
EXT_MPI_AMD_JOIN_TRACE=$PWD/$O/joinci.trace timeout -k 10 240 python3 bench.py --shape joinci > $O/joinci_trace.json 2> $O/joinci_trace.err || { tail -5 $O/joinci_trace.err; exit 1; }
for f in $O/joinci.trace.*; do python3 tools/join_trace_summary.py $f > $f.summary.txt; cat $f.summary.txt; done
port=29950
for N in 1 2; do
  port=$((port + 1))
  EXT_MPI_AMD_JOIN_PARTS=2 EXT_MPI_AMD_JOIN_TRACE=$PWD/$O/start_n$N.trace timeout -k 10 200 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $port bench.py --gpus $N --steps 20 --warmup 5 \
    --child-transport node-ipc --child-result $O/start_n${N}_r{rank}.json --child-deadline 150 > $O/start_n$N.log 2>&1 || { echo "n$N failed"; tail -5 $O/start_n$N.log; exit 1; }
  for f in $O/start_n$N.trace.*; do python3 tools/join_trace_summary.py $f > $f.summary.txt; echo "== $f"; cat $f.summary.txt; done
done
find $O -name "*.trace.[0-9]*" -size +8M -delete
exit 0
