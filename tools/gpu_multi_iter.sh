#!/bin/bash
# Multi-GPU paths rehearsed on one GPU: the ALS GPU tests (self-exchange, two ranks through IPC) and
# the MU exchange tests (k = 4 and 8).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/multi
mkdir -p $D
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_als.py -m gpu > $D/pytest_als.log 2>&1 &&
timeout -k 10 600 $T tests/test_gpu_exchange.py -m gpu > $D/pytest_exchange.log 2>&1
rc=$?
echo "exit=$rc"
exit $rc
