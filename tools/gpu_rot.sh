#!/bin/bash
# Rotated-window experiment: persistent-kernel tests, then the rotation probe with the default
# (non-temporal X loads) and the plain-load diagnostic library.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread"
timeout -k 10 500 $T tests/test_gpu_persistent.py tests/test_gpu_parity.py > gpurun_out/pytest_rot.log 2>&1 &&
timeout -k 10 300 python tools/rot_probe.py --mb 0,100,150,200,240 > gpurun_out/rot_nt.log 2>&1 &&
CNMF_HIP_LIB=$PWD/cnmf_amd/libcnmf_hip_plain.so timeout -k 10 300 python tools/rot_probe.py --mb 0,100,150,200,240 > gpurun_out/rot_plain.log 2>&1
echo "exit=$?"
