#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_als.py > gpurun_out/pytest_als.log 2>&1 &&
timeout -k 10 300 python bench.py --solver als --steps 100 --warmup 5 --no-cpu > gpurun_out/cfg5.log 2>&1 &&
CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_stamps.so timeout -k 10 200 python tools/timeline_persist.py > gpurun_out/timeline.log 2>&1
echo "exit=$?"
