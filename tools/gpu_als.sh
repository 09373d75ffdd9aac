#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_als.py > gpurun_out/pytest_als.log 2>&1 &&
timeout -k 10 600 $T tests -m gpu > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py --solver als --steps 100 --warmup 5 --cpu-seconds 10 > gpurun_out/cfg5.log 2>&1 &&
timeout -k 10 300 python bench.py --features 300 --k 16 --dtype bf16 --steps 100 --warmup 5 --no-cpu > gpurun_out/cfg4.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof5 -o run --output-format csv -- python3 bench.py --solver als --steps 30 --warmup 2 --no-cpu > gpurun_out/prof5.log 2>&1
echo "exit=$?"
