#!/bin/bash
# Layout 6 (reduce-scatter end of iteration): its GPU tests, then a same-box A/B against layout 4
# (cfg2, cfg3's shard, the N = 8 shard of cfg2) alternating the two.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/${1:-rs}
mkdir -p $D
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread"
B="timeout -k 10 200 python -u bench.py --no-cpu"
timeout -k 10 900 $T -m gpu tests/test_gpu_persistent.py tests/test_gpu_exchange.py tests/test_gpu_device_tol.py tests/test_gpu_cfg3.py -k "rs or 6" > $D/pytest_rs.log 2>&1 || exit 1
for r in 1 2; do
  for L in 4 6; do
    $B --layout $L > $D/cfg2_L${L}_$r.json 2> $D/cfg2_L${L}_$r.err || exit 1
    $B --layout $L --rows 124992 > $D/n8_L${L}_$r.json 2> $D/n8_L${L}_$r.err || exit 1
    $B --layout $L --rows 1250000 --k 8 > $D/k8_L${L}_$r.json 2> $D/k8_L${L}_$r.err || exit 1
  done
done
$B --layout 6 --steps 20 --warmup 5 > $D/cfg2_L6_driver.json 2> $D/cfg2_L6_driver.err || exit 1
echo "exit=0"
