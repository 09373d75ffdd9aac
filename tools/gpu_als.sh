#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_als.py > gpurun_out/pytest_als.log 2>&1 &&
timeout -k 10 600 $T tests -m gpu > gpurun_out/pytest_gpu.log 2>&1
echo "exit=$?"
