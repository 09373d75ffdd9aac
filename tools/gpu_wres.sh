#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_persistent.py > gpurun_out/pytest_persist.log 2>&1 &&
timeout -k 10 600 $T tests -m gpu > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu --steps 1000 > gpurun_out/bench_wres.log 2>&1 &&
CNMF_WRES=0 timeout -k 10 300 python bench.py --no-cpu --steps 1000 > gpurun_out/bench_nowres.log 2>&1 &&
CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_stamps.so timeout -k 10 200 python tools/timeline_persist.py > gpurun_out/timeline.log 2>&1
echo "exit=$?"
