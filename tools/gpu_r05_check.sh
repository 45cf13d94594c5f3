#!/bin/bash
# Round 5: chain parity tests, the default bench, then the chains' schedules forced (2 passes).
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05/check
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tuner.py -x -q -m gpu --timeout 300 \
  --timeout-method thread -k "leaf_major_chains or every_tuned or tuner or forced or tune" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 - <<'PY'
import json
d=json.load(open('gpurun_out/r05/check/bench.json'))
e=d['extras']
print('headline', d['ms_per_step'], d['roofline']['frac'], d['config']['fold_schedules_per_set'])
print('256', {k: e['point_256MiB'].get(k) for k in ('avg_launch_us','median_launch_us','min_launch_us','max_launch_us','launches_timed','frac_of_peak_at_median','schedules_per_set')})
print('local', {k: e['local_fold_256MiB'].get(k) for k in ('avg_launch_us','median_launch_us','min_launch_us','max_launch_us','frac_of_peak_at_median')})
print('chains', {k: (v['avg_launch_us'], v['vs_linear']) for k, v in e['radix_chains_16MiB'].items()})
print('int/long', e.get('config3_int_long_4MiB'))
PY
bash tools/gpu_r05_chains_ab.sh 524372,196626,1245202 2 final
