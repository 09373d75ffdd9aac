#!/bin/bash
# Timelines (stamps build) of layout 4 and layout 6 at cfg2, the N = 8 shard and cfg3's shard.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/${1:-rs_tl}
mkdir -p $D
export TMPDIR=/tmp PYTHONUNBUFFERED=1 CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_stamps.so
R="timeout -k 10 120 python -u tools/timeline_persist.py --iters 40"
for L in 4 6; do
  $R --layout $L > $D/tl_cfg2_L$L.log 2>&1 || exit 1
  $R --layout $L --rows 124992 > $D/tl_n8_L$L.log 2>&1 || exit 1
  $R --layout $L --rows 1250000 --k 8 > $D/tl_k8_L$L.log 2>&1 || exit 1
done
echo "exit=0"
