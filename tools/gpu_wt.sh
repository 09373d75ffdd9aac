#!/bin/bash
# wave-tile kernel: parity tests, then timings per layout / prefetch depth, and the compute floor
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_persistent.py tests/test_gpu_parity.py tests/test_gpu_exchange.py > gpurun_out/pytest_wt.log 2>&1 &&
timeout -k 10 200 python tools/rot_probe.py --mb 0 --variants 4,1 > gpurun_out/wt_pd3.log 2>&1 &&
CNMF_WT_PD=2 timeout -k 10 200 python tools/rot_probe.py --mb 0 --variants 4 > gpurun_out/wt_pd2.log 2>&1 &&
CNMF_WT_PD=4 timeout -k 10 200 python tools/rot_probe.py --mb 0 --variants 4 > gpurun_out/wt_pd4.log 2>&1 &&
CNMF_HIP_LIB=$PWD/cnmf_amd/libcnmf_hip_l2.so timeout -k 10 200 python tools/rot_probe.py --mb 0 --variants 4 > gpurun_out/wt_l2.log 2>&1
echo "exit=$?"
