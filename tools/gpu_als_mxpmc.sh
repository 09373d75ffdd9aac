#!/bin/bash
# cfg5 MX W-step (diag CNMF_ALS_OCC=7, ladder 2): SQ counter passes (each its own run, kernel-trace only)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/${1:-als_mxpmc}
mkdir -p $D
export TMPDIR=/tmp PYTHONUNBUFFERED=1 CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_diag.so CNMF_ALS_OCC=7 CNMF_ALS_PRIO=2
P="timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv"
A="--solver als --iters 20"
$P --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d $D/p1 -o p1 -- python3 tools/prof_pass.py $A > $D/p1.log 2>&1 &&
$P --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $D/p2 -o p2 -- python3 tools/prof_pass.py $A > $D/p2.log 2>&1 &&
$P --pmc SQ_INSTS_FLAT SQ_INSTS_VALU_FMA_F64 SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE GRBM_COUNT -d $D/p3 -o p3 -- python3 tools/prof_pass.py $A > $D/p3.log 2>&1
rc=$?
echo "exit=$rc"
exit $rc
