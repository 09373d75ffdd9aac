#!/bin/bash
# perf-iteration session: probe, parity tests, per-kernel timing (sample-lane vs VALU pass), bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 240 python tools/gpu_probe.py > gpurun_out/probe.log 2>&1 &&
timeout -k 10 600 python -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python tools/bench_pass.py > gpurun_out/bench_pass.log 2>&1 &&
CNMF_PASS_KERNEL=valu timeout -k 10 300 python tools/bench_pass.py > gpurun_out/bench_pass_valu.log 2>&1 &&
timeout -k 10 300 python tools/bench_pass.py --k 8 > gpurun_out/bench_pass_k8.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench.log 2>&1
echo "exit=$?"
