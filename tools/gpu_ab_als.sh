#!/bin/bash
# Same-box A/B of an ALS persistent-kernel change (cnmf_amd/libcnmf_hip_ab.so = before): the ALS
# GPU tests on the new build, then cfg5 bench lines old / new / old / new.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/ab_als
mkdir -p $D
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread"
B="timeout -k 10 300 python -u bench.py --solver als --no-cpu --steps 300 --warmup 100"
timeout -k 10 600 $T tests/test_gpu_als.py -m gpu > $D/pytest.log 2>&1 &&
CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_ab.so $B > $D/old.json 2> $D/e1 &&
$B > $D/new.json 2> $D/e2 &&
CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_ab.so $B > $D/old2.json 2> $D/e3 &&
$B > $D/new2.json 2> $D/e4
rc=$?
echo "exit=$rc"
exit $rc
