#!/bin/bash
# cfg5 A/B in the diagnostic build (same box, alternating): CNMF_ALS_OCC = 2 (the product kernel:
# two workgroups per CU), 4 (two per CU, phase 1 on the matrix cores), 5 (one per CU, matrix-core
# phase 1), 3 (one per CU, Hᵀ in VGPRs); then the ALS parity tests on variants 4 and 5.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
D=gpurun_out/${1:-als_ab}; mkdir -p $D
B="timeout -k 10 200 python -u bench.py --solver als --steps 200 --warmup 50 --no-cpu"
T="timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_diag.so CNMF_ALS_OCC=4 $T tests/test_gpu_als.py > $D/pytest_als_v4.log 2>&1 || exit 1
for r in 1 2; do
  for v in 2 4 5 3; do
    CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_diag.so CNMF_ALS_OCC=$v $B > $D/als_v${v}_r${r}.json 2> $D/als_v${v}_r${r}.err || exit 1
  done
done
CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_diag.so CNMF_ALS_OCC=5 $T tests/test_gpu_als.py > $D/pytest_als_v5.log 2>&1
echo "exit=$?"
