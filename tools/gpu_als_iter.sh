#!/bin/bash
# cfg5 iteration loop: ALS GPU parity tests, the stamps timeline (stream / tail / H-step, per-row
# BPP iterations and cycles), the cfg5 bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/als_iter
mkdir -p $D
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 180 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_als.py -m gpu > $D/pytest_als.log 2>&1 &&
CNMF_ALS_OCC=1 timeout -k 10 300 $T tests/test_gpu_als.py -m gpu -k persistent > $D/pytest_als_occ1.log 2>&1 &&
CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_stamps.so timeout -k 10 200 python tools/timeline_persist.py --solver als > $D/timeline.log 2>&1 &&
timeout -k 10 300 python -u bench.py --solver als --steps 200 --warmup 50 > $D/bench_als.json 2> $D/bench_als.err &&
CNMF_ALS_OCC=1 timeout -k 10 300 python -u bench.py --solver als --steps 200 --warmup 50 --no-cpu > $D/bench_als_occ1.json 2> $D/bench_als_occ1.err
rc=$?
echo "exit=$rc"
exit $rc
