#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/mall_probe.py > gpurun_out/mall_nt.log 2>&1 &&
CNMF_HIP_LIB=$PWD/cnmf_amd/libcnmf_hip_plain.so timeout -k 10 300 python tools/mall_probe.py > gpurun_out/mall_plain.log 2>&1
echo "exit=$?"
