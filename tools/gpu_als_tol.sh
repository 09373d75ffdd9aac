#!/bin/bash
# ALS device tolerance test: the ALS GPU tests, then the cfg5 bench at tol = 0 and 1e-4
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
D=gpurun_out/${1:-als_tol}; mkdir -p $D
T="timeout -k 10 500 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread"
$T tests/test_gpu_als.py tests/test_gpu_config_lengths.py -k "als or cfg5" > $D/pytest_als.log 2>&1 || exit 1
B="timeout -k 10 200 python -u bench.py --solver als --steps 200 --warmup 50 --no-cpu"
for r in 1 2; do
  $B > $D/als_r$r.json 2> $D/als_r$r.err || exit 1
  $B --tol 1e-4 > $D/als_tol_r$r.json 2> $D/als_tol_r$r.err || exit 1
done
echo "exit=0"
