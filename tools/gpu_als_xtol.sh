#!/bin/bash
# two-rank ALS exchange-plus-tolerance launch + the other ALS device-tol / exchange tests
set -o pipefail
mkdir -p gpurun_out/als_xtol
timeout -k 10 500 python -u -m pytest -x -v --timeout 420 --timeout-method thread tests/test_gpu_als.py \
  -k "two_ranks or device_tol" > gpurun_out/als_xtol/pytest.log 2>&1
