#!/bin/bash
# cfg4 counters and kernel time on one box, in-tree library (new) against cnmf_amd/libcnmf_hip_prev.so
# (prev): kernel-trace stats, then the MFMA / LDS counter passes of tools/gpu_evidence.sh.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/${1:-cfg4_pmc_ab}
mkdir -p $D
export TMPDIR=/tmp PYTHONUNBUFFERED=1
P="timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv"
C4="--rows 1000000 --features 300 --k 16 --dtype bf16 --iters 10"
B="bench.py --features 300 --k 16 --dtype bf16 --steps 100 --warmup 5 --no-cpu"
for v in new prev new2 prev2; do
  case $v in prev*) export CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_prev.so ;; *) unset CNMF_HIP_LIB ;; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_$v -o cfg4 --output-format csv -- python3 $B > $D/prof_$v.log 2>&1 || exit 1
done
for v in new prev; do
  case $v in prev) export CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_prev.so ;; *) unset CNMF_HIP_LIB ;; esac
  $P --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT -d $D/c4a_$v -o c4a -- python3 tools/prof_pass.py $C4 > $D/c4a_$v.log 2>&1 || exit 1
  $P --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY -d $D/c4b_$v -o c4b -- python3 tools/prof_pass.py $C4 > $D/c4b_$v.log 2>&1 || exit 1
done
echo "exit=0"
