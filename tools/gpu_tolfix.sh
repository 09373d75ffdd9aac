#!/bin/bash
# The device tolerance test's W snapshot counted in the prefetch waits: its tests, then the
# tol = 0 / tol = 1e-4 bench A/B on one box, and the k = 8 layouts' bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/${1:-tolfix}
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_device_tol.py tests/test_gpu_mf8.py tests/test_gpu_persistent.py > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -3 $D/pytest.log
B="timeout -k 10 240 python bench.py --no-cpu"
for r in 1 2; do
  $B --no-tune > $D/notune_$r.json 2> $D/e_notune_$r &&
  $B --no-tune --tol 1e-4 > $D/tol_$r.json 2> $D/e_tol_$r || exit 1
done
$B --rows 1250000 --k 8 --steps 200 --warmup 200 > $D/k8shard.json 2> $D/e_k8 || exit 1
for f in $D/*.json; do python - "$f" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d['roofline']
print(sys.argv[1].split('/')[-1], d['value'], r['avg_us_per_iteration_in_launch'], r['frac'], d['config'].get('tol_n_iter'), d['config'].get('layout_tuning_us_per_iteration'), d['config']['persistent_layout'][:30])
PY
done
