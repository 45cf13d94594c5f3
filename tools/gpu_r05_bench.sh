#!/bin/bash
# Round 5: the default bench (N = 1) alone, with a summary of the figures VERDICT r04 names.
# Usage: gpu_r05_bench.sh <tag>
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05/${1:-bench}
mkdir -p $O
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 - "$O/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); e = d['extras']
print('headline', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d.get('timing'))
for k in ('point_256MiB', 'local_fold_256MiB'):
    print(k, {f: e[k].get(f) for f in ('avg_launch_us', 'median_launch_us', 'min_launch_us', 'max_launch_us')})
print('chains', {k: (v['avg_launch_us'], v['vs_linear']) for k, v in e['radix_chains_16MiB'].items()})
print('int/long', e['config3_int_long_4MiB'])
print('sweep', [(x['bytes_per_rank'], x['us_per_allreduce']) for x in e['sweep_node_form']])
PY
