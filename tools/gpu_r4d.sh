#!/bin/bash
# cfg4 persistent (MFMA basis update, 16-B row stores): parity tests, bench, end-of-iteration stamps;
# cfg5: the MFL variant (matrix-core phase 1, B from LDS) A/B against the product kernel + its parity.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
D=gpurun_out/${1:-r4d}; mkdir -p $D
T="timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
$T tests/test_gpu_cfg4_persistent.py > $D/pytest_cfg4p.log 2>&1 &&
$T tests/test_gpu_device_tol.py tests/test_gpu_sharded_tol.py > $D/pytest_tol.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu > $D/bench_500.json 2> $D/bench_500.err &&
timeout -k 10 300 python -u bench.py --no-cpu --tol 1e-4 > $D/bench_tol.json 2> $D/bench_tol.err &&
timeout -k 10 300 python -u bench.py --features 300 --k 16 --dtype bf16 --steps 100 --warmup 10 --no-cpu > $D/bench_cfg4.json 2> $D/bench_cfg4.err &&
CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_stamps.so timeout -k 10 200 python -u tools/stamps_bfw_persist.py > $D/stamps_bfw_persist.log 2>&1 &&
CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_diag.so CNMF_ALS_OCC=6 $T tests/test_gpu_als.py > $D/pytest_als_v6.log 2>&1 || exit 1
B="timeout -k 10 200 python -u bench.py --solver als --steps 200 --warmup 50 --no-cpu"
for r in 1 2; do
  for v in 2 6; do
    CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_diag.so CNMF_ALS_OCC=$v $B > $D/als_v${v}_r${r}.json 2> $D/als_v${v}_r${r}.err || exit 1
  done
done
echo "exit=$?"
