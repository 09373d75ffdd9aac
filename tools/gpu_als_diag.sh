#!/bin/bash
# cfg5 diagnostics: the persistent constrained-ALS launch's timeline from the stamps build (stream /
# tail / H-step per iteration, BPP iterations and cycles per basis row), then SQ counter passes of
# als_iter_wt_kernel (each its own run, kernel-trace only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/${1:-als_diag}
mkdir -p $D
export TMPDIR=/tmp PYTHONUNBUFFERED=1
P="timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv"
A="--solver als --iters 20"
CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_stamps.so timeout -k 10 200 python tools/timeline_persist.py --solver als > $D/timeline.log 2>&1 &&
$P --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d $D/p1 -o p1 -- python3 tools/prof_pass.py $A > $D/p1.log 2>&1 &&
$P --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $D/p2 -o p2 -- python3 tools/prof_pass.py $A > $D/p2.log 2>&1 &&
$P --pmc SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_TRANS_F64 SQ_INST_CYCLES_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_FMA_F64 GRBM_GUI_ACTIVE GRBM_COUNT -d $D/p3 -o p3 -- python3 tools/prof_pass.py $A > $D/p3.log 2>&1
rc=$?
echo "exit=$rc"
exit $rc
