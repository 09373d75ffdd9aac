#!/bin/bash
# Same-box A/B of the batched resume loads (cnmf_amd/libcnmf_hip_ab.so = before): persistent / cfg3 /
# ALS / weighted GPU tests on the new build, then cfg2, cfg3 shard and cfg5 lines old / new twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/ab_resume
mkdir -p $D
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread"
B="timeout -k 10 300 python -u bench.py --no-cpu --no-tune"
O="env CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_ab.so"
timeout -k 10 700 $T tests/test_gpu_persistent.py tests/test_gpu_cfg3.py tests/test_gpu_als.py tests/test_gpu_wmu.py -m gpu > $D/pytest.log 2>&1 &&
CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_ab.so $B --steps 500 --warmup 500 > $D/old_cfg2.json 2> $D/e1 &&
$B --steps 500 --warmup 500 > $D/new_cfg2.json 2> $D/e2 &&
CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_ab.so $B --rows 1250000 --k 8 --steps 500 --warmup 500 > $D/old_cfg3shard.json 2> $D/e3 &&
$B --rows 1250000 --k 8 --steps 500 --warmup 500 > $D/new_cfg3shard.json 2> $D/e4 &&
CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_ab.so $B --steps 500 --warmup 500 > $D/old2_cfg2.json 2> $D/e5 &&
$B --steps 500 --warmup 500 > $D/new2_cfg2.json 2> $D/e6 &&
CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_ab.so $B --solver als --steps 300 --warmup 100 > $D/old_cfg5.json 2> $D/e7 &&
$B --solver als --steps 300 --warmup 100 > $D/new_cfg5.json 2> $D/e8
rc=$?
echo "exit=$rc"
exit $rc
