#!/bin/bash
# Round 6: the local fold's lease fingerprint, appended to each GPU call of the
# round, so slow and fast leases can be told apart by counter. The local fold (8 x 32 MiB -> 1,
# bench.py --shape local256: 40 launches of the tuned handle, per-launch events) timed, the read
# ceiling streams of the same lease (bench.py --shape copy256's phased copy), then rocprofv3 PMC
# passes of the fold: memory-side read requests and their cycles in flight, DRAM credit stalls.
# Usage: gpu_r06_localfp.sh <tag>
cd "$GRAFT_REPO_ROOT"
R=$PWD
O=gpurun_out/r06/localfp/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 5 60 python3 -c "
import torch
p = torch.cuda.get_device_properties(0)
print('uuid', getattr(p, 'uuid', '?'), 'pci', getattr(p, 'pci_bus_id', '?'), getattr(p, 'pci_device_id', '?'))" > $O/host.txt 2>/dev/null
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --shape local256 > $O/time_local256_$i.json 2> $O/time_local256_$i.err || exit $?
  echo "localfp $1 local256 pass $i: $(cat $O/time_local256_$i.json)"
done
pass() {  # group counters...
  local group=$1; shift
  rm -rf $O/local256_$group
  timeout -s KILL 180 rocprofv3 --pmc "$@" -d $R/$O/local256_$group -o run --output-format csv -- \
    python3 $R/bench.py --shape local256 > $O/local256_$group.json 2> $O/local256_$group.err
  local rc=$?
  echo "localfp pmc $group rc=$rc"
  if [ $rc -eq 137 ] || [ $rc -eq 124 ]; then exit $rc; fi
  return 0
}
pass level TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE
pass stall TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE
python3 tools/pmc_counters.py --by-kernel $O/local256_level $O/local256_stall > $O/pmc_local.json
for f in $(find $O -name "*counter_collection*.csv"); do rm -f $f; done  # the medians above are kept
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
t = [json.loads(open(f"{o}/time_local256_{i}.json").read()) for i in (1, 2)]
p = json.load(open(f"{o}/pmc_local.json"))
row = {"avg_launch_us": [x.get("avg_launch_us") for x in t], "median_launch_us": [x.get("median_launch_us") for x in t],
       "schedule": [x.get("schedule") for x in t]}
for d, ks in p.items():
    for k, c in ks.items():
        if "RDREQ_LEVEL" in str(c):
            row[k] = {"read_cycles_in_flight_per_request": round(c["TCC_EA0_RDREQ_LEVEL_sum"] / c["TCC_EA0_RDREQ_sum"], 1)}
for d, ks in p.items():
    for k, c in ks.items():
        if "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum" in c:
            row.setdefault(k, {})["dram_write_credit_stall_per_write_req"] = round(
                c["TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum"] / max(1, c["TCC_EA0_WRREQ_sum"]), 3)
json.dump(row, open(f"{o}/summary.json", "w"), indent=1)
print("localfp summary", json.dumps(row))
PY
exit 0
