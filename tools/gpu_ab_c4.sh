#!/bin/bash
# Same-box A/B for the k > 4 basis update (cnmf_amd/libcnmf_hip_ab.so = before): bf16 / k8 parity
# tests on the new build, cfg4 bench lines old / new / old / new, kernel stats of the new one.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/ab_c4
mkdir -p $D
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread"
B="timeout -k 10 300 python -u bench.py --features 300 --k 16 --dtype bf16 --steps 100 --warmup 10 --no-cpu"
timeout -k 10 600 $T tests/test_gpu_parity.py -m gpu > $D/pytest.log 2>&1 &&
CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_ab.so $B > $D/old.json 2> $D/e1 &&
$B > $D/new.json 2> $D/e2 &&
CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_ab.so $B > $D/old2.json 2> $D/e3 &&
$B > $D/new2.json 2> $D/e4 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/p -o c4 --output-format csv -- python3 bench.py --features 300 --k 16 --dtype bf16 --steps 50 --warmup 5 --no-cpu --no-tune > $D/prof.log 2>&1
rc=$?
echo "exit=$rc"
exit $rc
