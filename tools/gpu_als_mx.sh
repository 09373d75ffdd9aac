#!/bin/bash
# cfg5: the matrix-core W-step (MX: diag CNMF_ALS_OCC=7 two workgroups per CU, =8 one) — parity, then
# the A/B against the product kernel, two rounds.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
D=gpurun_out/${1:-als_mx}; mkdir -p $D
T="timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread"
CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_diag.so CNMF_ALS_OCC=8 $T tests/test_gpu_als.py > $D/pytest_als_v8.log 2>&1 || exit 1
CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_diag.so CNMF_ALS_OCC=7 $T tests/test_gpu_als.py > $D/pytest_als_v7.log 2>&1 || exit 1
B="timeout -k 10 200 python -u bench.py --solver als --steps 200 --warmup 50 --no-cpu"
for r in 1 2; do
  for v in 2 7 8; do
    CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_diag.so CNMF_ALS_OCC=$v $B > $D/als_v${v}_r$r.json 2> $D/als_v${v}_r$r.err || exit 1
  done
done
echo "exit=0"
