#!/bin/bash
# Floating-tile layout (variant 3): its parity tests, then the bench (which times all layouts) at three fractions.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_persistent.py -m gpu > gpurun_out/pytest_persist.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_dyn.log 2>&1 &&
CNMF_DYN_FRAC=0.7 timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_dyn07.log 2>&1 &&
CNMF_DYN_FRAC=0.9 timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_dyn09.log 2>&1
echo "exit=$?"
