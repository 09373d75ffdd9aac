#!/bin/bash
# persistent-kernel session: its parity tests first, then the full GPU suite, then bench A/B
# (persistent PD=2 / PD=1 / per-iteration launches) and a kernel-trace profile of the bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_persistent.py > gpurun_out/pytest_persist.log 2>&1 &&
timeout -k 10 600 $T tests -m gpu > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_pd2.log 2>&1 &&
CNMF_PERSIST_PD=1 timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_pd1.log 2>&1 &&
CNMF_PERSIST=0 timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_nopersist.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 500 --no-cpu > gpurun_out/prof.log 2>&1
echo "exit=$?"
