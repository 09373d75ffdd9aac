#!/bin/bash
# Weighted / masked MU: parity tests, then a timing of the cfg2-shaped weighted pass.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_wmu.py -m gpu > gpurun_out/pytest_wmu.log 2>&1 &&
timeout -k 10 300 python bench.py --weighted --no-cpu --steps 100 --warmup 20 > gpurun_out/bench_wmu.log 2>&1
echo "exit=$?"
