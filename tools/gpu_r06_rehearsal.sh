#!/bin/bash
# Round 6: the exact N > 1 command the driver runs on an 8-GPU node --
# torchrun --nproc-per-node 8 bench.py --gpus 8 --steps 20 --warmup 5, default deadline
# (bench.py MULTI_DEADLINE_S) -- rehearsed with the 8 processes sharing the one MI355X. Records the
# wall time, the line, and a summary (headline transport and check, the one-rank-per-GPU child's
# sweep incl. configs[3]'s double 256 MiB, the failures). Usage: gpu_r06_rehearsal.sh [N]
cd "$GRAFT_REPO_ROOT"
N=${1:-8}
O=gpurun_out/r06/rehearsal
mkdir -p $O
t0=$(date +%s)
timeout -k 10 1170 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
  --master-port 29640 bench.py --gpus $N --steps 20 --warmup 5 > $O/bench_n$N.json 2> $O/bench_n$N.err
rc=$?
t1=$(date +%s)
echo "rehearsal n=$N rc=$rc wall_s=$((t1 - t0))" | tee $O/wall_n$N.txt
[ $rc -ne 0 ] && { tail -30 $O/bench_n$N.err; exit $rc; }
python3 - $O/bench_n$N.json $((t1 - t0)) <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d.get("extras", {})
print("value", d["value"], "ms_per_step", d["ms_per_step"], "transport", d["config"].get("transport"),
      "checked", d["config"].get("checked_vs_fp64_sum"), "join_parts", e.get("join_parts"), "wall_s", sys.argv[2])
print("parts_us", e.get("parts_us"))
o = e.get("one_rank_per_gpu", {})
oe = o.get("extras", {}) if isinstance(o, dict) else {}
print("one_rank_per_gpu:", o.get("config", {}).get("transport"), "checked", o.get("config", {}).get("checked_vs_fp64_sum"))
for p in oe.get("sweep", []):
    print("  sweep", p)
print("  radix_crossover", oe.get("radix_crossover"))
print("failures", [(f.get("transport"), f.get("rank"), f.get("rc"), f.get("error")) for f in e.get("failures", [])])
PY
