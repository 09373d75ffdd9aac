#!/bin/bash
# cfg5 MX (diag CNMF_ALS_OCC=7): timelines with and without the priority ladder, A/B with the ladder
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
D=gpurun_out/${1:-als_mx2}; mkdir -p $D
CNMF_ALS_OCC=7 CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_stamps.so timeout -k 10 200 python tools/timeline_persist.py --solver als > $D/timeline_v7.log 2>&1 &&
CNMF_ALS_OCC=7 CNMF_ALS_PRIO=4 CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_stamps.so timeout -k 10 200 python tools/timeline_persist.py --solver als > $D/timeline_v7p4.log 2>&1 || exit 1
B="timeout -k 10 200 python -u bench.py --solver als --steps 200 --warmup 50 --no-cpu"
for r in 1 2; do
  for p in 0 2 4; do
    CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_diag.so CNMF_ALS_OCC=7 CNMF_ALS_PRIO=$p $B > $D/als_v7p${p}_r$r.json 2> $D/als_v7p${p}_r$r.err || exit 1
  done
done
echo "exit=0"
