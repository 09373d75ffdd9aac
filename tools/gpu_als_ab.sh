#!/bin/bash
# cfg5 (constrained ALS) A/B on one box: the in-tree library against cnmf_amd/libcnmf_hip_prev.so
# (a build of the previous source), alternating bench runs; ALS GPU tests on the in-tree library first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/${1:-als_ab}
mkdir -p $D
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -s -p no:cacheprovider --timeout 600 --timeout-method thread"
timeout -k 10 900 $T -m gpu tests/test_gpu_als.py > $D/pytest.log 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py --solver als --steps 200 --warmup 50 --no-cpu > $D/new_$r.json 2> $D/new_$r.err || exit 1
  [ -f cnmf_amd/libcnmf_hip_prev.so ] || continue
  CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_prev.so timeout -k 10 300 python -u bench.py --solver als --steps 200 --warmup 50 --no-cpu > $D/prev_$r.json 2> $D/prev_$r.err || exit 1
done
echo "exit=0"
