#!/bin/bash
# Round-4 A/B: an event recorded after every fold launch (EXT_MPI_AMD_FOLD_FENCE: 0 none, 1 the
# default event's system-scope fence, 2 a release to system scope) -- the profiled bench command
# ran the 256 MiB point at 694 us where the unprofiled one ran it at 751 us on the same lease.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/fence4
mkdir -p $O
for rep in 1 2; do
  for shape in node256 node16 node64; do
    for f in 0 1 2; do
      EXT_MPI_AMD_FOLD_FENCE=$f timeout -k 10 240 python3 bench.py --shape $shape > $O/${shape}_f${f}_$rep.json 2> $O/${shape}_f${f}_$rep.err || { echo "$shape $f rc=$?"; tail -3 $O/${shape}_f${f}_$rep.err; exit 1; }
      echo "$rep $shape fence=$f $(cat $O/${shape}_f${f}_$rep.json)"
    done
  done
done
exit 0
