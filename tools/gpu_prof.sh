#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp PYTHONUNBUFFERED=1
P="timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv"
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_persistent.py > gpurun_out/pytest_persist.log 2>&1 &&
$P --pmc FETCH_SIZE -d gpurun_out/pmc/fetch -o fetch -- python3 tools/prof_pass.py > gpurun_out/pmc/fetch.log 2>&1 &&
$P --pmc WRITE_SIZE -d gpurun_out/pmc/write -o write -- python3 tools/prof_pass.py > gpurun_out/pmc/write.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 500 --warmup 500 --no-cpu > gpurun_out/prof.log 2>&1
echo "exit=$?"
