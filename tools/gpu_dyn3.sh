#!/bin/bash
# Floating tiles: probe timings, then the persistent parity tests (all layouts).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread"
timeout -k 10 300 python tools/dyn_probe.py > gpurun_out/dyn_probe.log 2>&1 &&
timeout -k 10 400 $T tests/test_gpu_persistent.py -m gpu > gpurun_out/pytest_persist.log 2>&1
echo "exit=$?"
