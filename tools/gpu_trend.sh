#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
(rocm-smi --showclocks --showtemp --showpower > gpurun_out/smi_before.log 2>&1 || true)
timeout -k 10 300 python tools/bench_trend.py > gpurun_out/trend.log 2>&1 &&
(rocm-smi --showclocks --showtemp --showpower > gpurun_out/smi_after.log 2>&1 || true) &&
GAP=2 REPS=5 timeout -k 10 300 python tools/bench_trend.py > gpurun_out/trend_gap.log 2>&1 &&
CNMF_WRES=0 REPS=5 timeout -k 10 300 python tools/bench_trend.py > gpurun_out/trend_nowres.log 2>&1
echo "exit=$?"
