#!/bin/bash
# PMC counter passes (kernel-trace only, no sys/hip trace; one counter group per pass)
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp PYTHONUNBUFFERED=1
P="timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv"
$P --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d gpurun_out/pmc/p1 -o p1 -- python3 tools/prof_pass.py > gpurun_out/pmc/p1.log 2>&1 &&
$P --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d gpurun_out/pmc/p2 -o p2 -- python3 tools/prof_pass.py > gpurun_out/pmc/p2.log 2>&1 &&
$P --pmc FETCH_SIZE -d gpurun_out/pmc/p3 -o p3 -- python3 tools/prof_pass.py > gpurun_out/pmc/p3.log 2>&1 &&
$P --pmc WRITE_SIZE -d gpurun_out/pmc/p4 -o p4 -- python3 tools/prof_pass.py > gpurun_out/pmc/p4.log 2>&1 &&
$P --pmc SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc/p5 -o p5 -- python3 tools/prof_pass.py > gpurun_out/pmc/p5.log 2>&1
echo "exit=$?"
