#!/bin/bash
# The device tolerance test: its GPU tests, then tol = 0 against tol = 1e-4 alternating on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/${1:-tol_ab}
mkdir -p $D
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 600 $T -m gpu tests/test_gpu_device_tol.py tests/test_gpu_mf8.py > $D/pytest.log 2>&1 || exit 1
B="timeout -k 10 200 python -u bench.py --no-cpu --no-tune"
for r in 1 2; do
  $B > $D/tol0_$r.json 2> $D/tol0_$r.err || exit 1
  $B --tol 1e-4 > $D/tol_$r.json 2> $D/tol_$r.err || exit 1
done
echo "exit=0"
