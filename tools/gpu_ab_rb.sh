#!/bin/bash
# Same-box A/B of the reduction batch change (cnmf_amd/libcnmf_hip_ab.so = before): k = 8 and
# weighted GPU tests on the new build, then cfg3 shard and weighted bench lines, old and new.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/ab_rb
mkdir -p $D
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread"
B="timeout -k 10 300 python -u bench.py --no-cpu"
timeout -k 10 600 $T tests/test_gpu_cfg3.py tests/test_gpu_wmu.py -m gpu > $D/pytest.log 2>&1 &&
CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_ab.so $B --rows 1250000 --k 8 --steps 500 --warmup 500 > $D/old_cfg3shard.json 2> $D/e1 &&
$B --rows 1250000 --k 8 --steps 500 --warmup 500 > $D/new_cfg3shard.json 2> $D/e2 &&
CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_ab.so $B --weighted --steps 200 --warmup 50 > $D/old_weighted.json 2> $D/e3 &&
$B --weighted --steps 200 --warmup 50 > $D/new_weighted.json 2> $D/e4 &&
CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_ab.so $B --rows 1250000 --k 8 --steps 500 --warmup 500 > $D/old2_cfg3shard.json 2> $D/e5 &&
$B --rows 1250000 --k 8 --steps 500 --warmup 500 > $D/new2_cfg3shard.json 2> $D/e6
rc=$?
echo "exit=$rc"
exit $rc
