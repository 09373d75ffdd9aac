#!/bin/bash
# same-box A/B: the product library vs the diagnostic build of a candidate source (CNMF_HIP_LIB)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
D=gpurun_out/${1:-als_ab3}; mkdir -p $D
B="timeout -k 10 200 python -u bench.py --solver als --steps 200 --warmup 50 --no-cpu"
for r in 1 2 3; do
  $B > $D/prod_r$r.json 2> $D/prod_r$r.err || exit 1
  CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_diag.so $B > $D/cand_r$r.json 2> $D/cand_r$r.err || exit 1
done
CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_diag.so timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_als.py -k "persistent" > $D/pytest_cand.log 2>&1
rc=$?; echo "exit=$rc"; exit $rc
