#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_parity.py -k "bf16" > gpurun_out/pytest_bf16.log 2>&1 &&
timeout -k 10 300 python bench.py --features 300 --k 16 --dtype bf16 --steps 100 --warmup 5 --no-cpu > gpurun_out/cfg4.log 2>&1 &&
timeout -k 10 600 $T tests -m gpu > gpurun_out/pytest_gpu.log 2>&1
echo "exit=$?"
