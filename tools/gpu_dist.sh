#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python bench.py --no-cpu --dist > gpurun_out/bench_dist.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profd -o run --output-format csv -- python3 bench.py --no-cpu --dist --steps 200 --warmup 200 > gpurun_out/profd.log 2>&1
echo "exit=$?"
