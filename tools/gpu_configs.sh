#!/bin/bash
# every BASELINE.json config on one GPU: cfg2 (headline), cfg5 (ALS), cfg4 (bf16 F=300 k=16),
# cfg3's per-GPU shard (1.25e6 x 81, k=8), and the weighted MU on the cfg2 shape
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/cfg2.log 2>&1 &&
timeout -k 10 300 python bench.py --solver als --steps 100 --warmup 5 --cpu-seconds 10 > gpurun_out/cfg5.log 2>&1 &&
timeout -k 10 300 python bench.py --features 300 --k 16 --dtype bf16 --steps 100 --warmup 5 --no-cpu > gpurun_out/cfg4.log 2>&1 &&
timeout -k 10 300 python bench.py --rows 1250000 --k 8 --steps 200 --warmup 10 --no-cpu > gpurun_out/cfg3shard.log 2>&1 &&
timeout -k 10 300 python bench.py --weighted --steps 100 --warmup 20 --no-cpu > gpurun_out/weighted.log 2>&1
echo "exit=$?"
