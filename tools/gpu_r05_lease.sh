#!/bin/bash
# Round 5: a fingerprint of the lease for the 256 MiB point. On every lease
# it runs, the same measurements: the 256 MiB node launch under its usual kept schedule (U 4 burst,
# buffer loads, device-scope stores: word 49153 << 4 | 4) and leaf-major groups, timed; the 1:1
# copies of its 4 GiB; then rocprofv3 PMC passes (one counter group per run) of both: memory-side
# requests, DRAM credit stalls, in-flight levels. Slow and fast leases are then told apart by
# counter (tools/lease_compare.py over every fingerprint collected).
# Usage: gpu_r05_lease.sh <tag>
cd "$GRAFT_REPO_ROOT"
R=$PWD
O=gpurun_out/r05/lease/$1
mkdir -p $O
export TMPDIR=/tmp
W=786452,196626  # (4 | (1 | kDevStore | kBufLoad) << 4), leaf-major (U 2, 4 tiles)
# which GPU (uuid, PCI location) and its clocks at the time (read-only queries)
timeout -k 5 60 python3 -c "
import torch
p = torch.cuda.get_device_properties(0)
print('uuid', getattr(p, 'uuid', '?'), 'pci', getattr(p, 'pci_bus_id', '?'), getattr(p, 'pci_device_id', '?'),
      'cus', p.multi_processor_count, 'mem', p.total_memory)" > $O/host.txt 2>/dev/null
timeout -k 5 60 rocm-smi --showclocks >> $O/host.txt 2>&1 || true
timeout -k 10 300 python3 bench.py --shape node256 --schedules $W > $O/time_node256.json 2> $O/time_node256.err || exit $?
echo "time node256 $(cat $O/time_node256.json)"
# the kept schedule's launches back to back and each alone (the host waits between them)
# ... and on 4 more freshly allocated buffer sets (the placement inside one lease)
EXT_MPI_AMD_FOLD_SCHEDULE=786452 EXT_MPI_AMD_BENCH_ISOLATED=1 EXT_MPI_AMD_BENCH_PLACEMENTS=4 EXT_MPI_AMD_BENCH_FAST_FILL=1 \
  timeout -k 10 400 python3 bench.py --shape node256 > $O/time_node256_iso.json 2> $O/time_node256_iso.err || exit $?
echo "time node256 back to back / isolated $(cat $O/time_node256_iso.json)"
timeout -k 10 300 python3 bench.py --shape copy256 > $O/time_copy256.json 2> $O/time_copy256.err || exit $?
echo "time copy256 $(cat $O/time_copy256.json)"
pass() {  # shape group counters...
  local shape=$1 group=$2; shift 2
  local extra=""
  [ "$shape" = node256 ] && extra="--schedules 786452"
  rm -rf $O/${shape}_$group
  timeout -s KILL 240 rocprofv3 --pmc "$@" -d $R/$O/${shape}_$group -o run --output-format csv -- \
    python3 $R/bench.py --shape $shape $extra > $O/${shape}_$group.json 2> $O/${shape}_$group.err
  local rc=$?
  echo "pmc $shape $group rc=$rc"
  if [ $rc -eq 137 ] || [ $rc -eq 124 ]; then exit $rc; fi
  [ $rc -ne 0 ] && tail -n 3 $O/${shape}_$group.err
  return 0
}
for shape in node256 copy256; do
  pass $shape ea TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum GRBM_GUI_ACTIVE
  pass $shape stall TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum GRBM_GUI_ACTIVE
  pass $shape level TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_LEVEL_sum GRBM_GUI_ACTIVE
done
python3 tools/pmc_counters.py --by-kernel $O/node256_* > $O/pmc_fold.json
python3 tools/pmc_counters.py --by-kernel --kernel='copy_k4|copy_phased' $O/copy256_* > $O/pmc_copy.json
# keep the fold's and the copies' rows only (the bench's fill kernels make the files large)
for f in $(find $O -name "*counter_collection*.csv"); do
  python3 -c "
import sys
rows = open(sys.argv[1]).read().splitlines()
open(sys.argv[1], 'w').write('\n'.join(rows[:1] + [r for r in rows[1:] if 'fold_' in r or 'copy_' in r]) + '\n')" $f
done
python3 tools/lease_compare.py gpurun_out/r05/lease
exit 0
