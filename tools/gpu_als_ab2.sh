#!/bin/bash
# same-box A/B: the cfg5 ALS of the previous commit's library (libcnmf_hip_head.so) vs the current
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
D=gpurun_out/${1:-als_ab2}; mkdir -p $D
B="timeout -k 10 200 python -u bench.py --solver als --steps 200 --warmup 50 --no-cpu"
for r in 1 2; do
  CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_head.so $B > $D/head_r$r.json 2> $D/head_r$r.err || exit 1
  $B > $D/cur_r$r.json 2> $D/cur_r$r.err || exit 1
done
echo "exit=0"
