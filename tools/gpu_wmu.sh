#!/bin/bash
# Weighted / masked MU: parity tests, then timings of the cfg2-shaped weighted fit (the persistent
# launch, and the per-iteration kernels with CNMF_WMU_PERSIST=0), then the kernel-trace stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 180 --timeout-method thread"
timeout -k 10 500 $T tests/test_gpu_wmu.py -m gpu > gpurun_out/pytest_wmu.log 2>&1 &&
timeout -k 10 300 python bench.py --weighted --no-cpu --steps 200 --warmup 50 > gpurun_out/bench_wmu.log 2>&1 &&
CNMF_WMU_PERSIST=0 timeout -k 10 300 python bench.py --weighted --no-cpu --steps 100 --warmup 20 > gpurun_out/bench_wmu_pass.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wmu -o run --output-format csv -- python3 bench.py --weighted --no-cpu --steps 200 --warmup 50 > gpurun_out/prof_wmu.log 2>&1
echo "exit=$?"
