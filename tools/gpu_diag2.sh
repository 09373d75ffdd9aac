#!/bin/bash
# Diagnostics from the stamps build: per-phase cycles of the cfg4 bf16 MFMA pass, and the timeline
# of cfg3's k = 8 shard (1.25e6 rows) in the persistent wave-tile launch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/diag2
mkdir -p $D
export TMPDIR=/tmp PYTHONUNBUFFERED=1
CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_stamps.so timeout -k 10 300 python -u tools/stamps_bf16.py > $D/stamps_bf16.log 2>&1 &&
CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_stamps.so timeout -k 10 200 python -u tools/timeline_persist.py --rows 1250000 --k 8 > $D/timeline_k8.log 2>&1
rc=$?
echo "exit=$rc"
exit $rc
