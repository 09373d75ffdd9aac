#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_parity.py -k "bf16" > gpurun_out/pytest_bf16.log 2>&1 &&
timeout -k 10 600 $T tests -m gpu > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py --features 300 --k 16 --dtype bf16 --steps 100 --warmup 5 --no-cpu > gpurun_out/cfg4.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4 -o run --output-format csv -- python3 bench.py --features 300 --k 16 --dtype bf16 --steps 30 --warmup 2 --no-cpu > gpurun_out/prof4.log 2>&1
echo "exit=$?"
B="python3 bench.py --features 300 --k 16 --dtype bf16 --steps 30 --warmup 2 --no-cpu"
mkdir -p gpurun_out/pmc4
P="timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv"
$P --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES -d gpurun_out/pmc4/p2 -o p2 -- $B > gpurun_out/pmc4/p2.log 2>&1
echo "exit2=$?"
