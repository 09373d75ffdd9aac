#!/bin/bash
# SQ counter passes of the persistent kernel (each its own run; kernel-trace only)
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp PYTHONUNBUFFERED=1
P="timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv"
A="--iters ${ITERS:-200}"
$P --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d gpurun_out/pmc/p1 -o p1 -- python3 tools/prof_pass.py $A > gpurun_out/pmc/p1.log 2>&1 &&
$P --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d gpurun_out/pmc/p2 -o p2 -- python3 tools/prof_pass.py $A > gpurun_out/pmc/p2.log 2>&1 &&
$P --pmc SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmc/p5 -o p5 -- python3 tools/prof_pass.py $A > gpurun_out/pmc/p5.log 2>&1
echo "exit=$?"
