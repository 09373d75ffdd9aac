#!/bin/bash
# cfg5 product: ALS parity, timeline (H-step phases), bench x2
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
D=gpurun_out/${1:-als_hs}; mkdir -p $D
T="timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread"
$T tests/test_gpu_als.py tests/test_gpu_config_lengths.py -k "als or cfg5" > $D/pytest_als.log 2>&1 || exit 1
CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_stamps.so timeout -k 10 200 python tools/timeline_persist.py --solver als > $D/timeline.log 2>&1 || exit 1
B="timeout -k 10 200 python -u bench.py --solver als --steps 200 --warmup 50 --no-cpu"
for r in 1 2; do
  $B > $D/als_r$r.json 2> $D/als_r$r.err || exit 1
done
echo "exit=0"
