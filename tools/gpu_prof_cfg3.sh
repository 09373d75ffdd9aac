#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/pmc3
export TMPDIR=/tmp PYTHONUNBUFFERED=1
B="python3 bench.py --rows 1250000 --k 8 --steps 30 --warmup 30 --no-cpu"
P="timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv"
$P --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC -d gpurun_out/pmc3/p1 -o p1 -- $B > gpurun_out/pmc3/p1.log 2>&1 &&
$P --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES -d gpurun_out/pmc3/p2 -o p2 -- $B > gpurun_out/pmc3/p2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o run --output-format csv -- $B > gpurun_out/prof3.log 2>&1
echo "exit=$?"
