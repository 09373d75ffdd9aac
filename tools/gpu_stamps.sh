#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_stamps.so CNMF_FORCE_VALU=1 timeout -k 10 300 python tools/stamps_pass.py > gpurun_out/stamps.log 2>&1 &&
K=8 CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_stamps.so CNMF_FORCE_VALU=1 timeout -k 10 300 python tools/stamps_pass.py > gpurun_out/stamps_k8.log 2>&1
echo "exit=$?"
