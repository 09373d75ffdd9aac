#!/bin/bash
# Counter passes (each its own run, kernel-trace only, <= 8 SQ / 4 TCC / 2 GRBM counters):
#   k8  — cfg3's shard (1.25e6 x 81, k = 8, the wave-tile kernel with W streamed): issue / wait /
#         instruction mix, and HBM traffic (FETCH_SIZE, WRITE_SIZE);
#   cfg4 — 1e6 x 300 bf16, k = 16 (mu_pass_bf16_mfma_kernel): MFMA busy / MOPS per type and LDS
#         bank conflicts.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/pmc_cfg
export TMPDIR=/tmp PYTHONUNBUFFERED=1
P="timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv"
K8="--rows 1250000 --k 8 --iters 20"
C4="--rows 1000000 --features 300 --k 16 --dtype bf16 --iters 10"
D=gpurun_out/pmc_cfg
$P --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d $D/k8a -o k8a -- python3 tools/prof_pass.py $K8 > $D/k8a.log 2>&1 &&
$P --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $D/k8b -o k8b -- python3 tools/prof_pass.py $K8 > $D/k8b.log 2>&1 &&
$P --pmc FETCH_SIZE -d $D/k8f -o k8f -- python3 tools/prof_pass.py $K8 > $D/k8f.log 2>&1 &&
$P --pmc WRITE_SIZE -d $D/k8w -o k8w -- python3 tools/prof_pass.py $K8 > $D/k8w.log 2>&1 &&
$P --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT -d $D/c4a -o c4a -- python3 tools/prof_pass.py $C4 > $D/c4a.log 2>&1 &&
$P --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU_MFMA_BF16 SQ_INSTS_VALU_MFMA_F64 SQ_WAIT_INST_ANY -d $D/c4b -o c4b -- python3 tools/prof_pass.py $C4 > $D/c4b.log 2>&1
echo "exit=$?"
