#!/bin/bash
# End-of-iteration variants of the wave-tile kernel: layout 4 (ticket tree + flag), 7 (tree, AB as
# tagged granules), 6 (reduce-scatter): timelines (stamps build), a same-box A/B of the product
# build (cfg2, the N = 8 shard, cfg3's shard), then the tests of 6 / 7.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/${1:-sync_ab}
mkdir -p $D
export TMPDIR=/tmp PYTHONUNBUFFERED=1
R="timeout -k 10 120 python -u tools/timeline_persist.py --iters 40"
for L in 4 7 6; do
  CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_stamps.so $R --layout $L > $D/tl_cfg2_L$L.log 2>&1 || exit 1
  CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_stamps.so $R --layout $L --rows 124992 > $D/tl_n8_L$L.log 2>&1 || exit 1
done
B="timeout -k 10 200 python -u bench.py --no-cpu"
for r in 1 2; do
  for L in 4 7 6; do
    $B --layout $L > $D/cfg2_L${L}_$r.json 2> $D/cfg2_L${L}_$r.err || exit 1
    $B --layout $L --rows 124992 > $D/n8_L${L}_$r.json 2> $D/n8_L${L}_$r.err || exit 1
    $B --layout $L --rows 1250000 --k 8 > $D/k8_L${L}_$r.json 2> $D/k8_L${L}_$r.err || exit 1
  done
done
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 900 $T -m gpu tests/test_gpu_persistent.py tests/test_gpu_exchange.py tests/test_gpu_device_tol.py tests/test_gpu_cfg3.py -k "rs or tab or 6 or 7" > $D/pytest_sync.log 2>&1 || exit 1
echo "exit=0"
