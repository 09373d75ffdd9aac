#!/bin/bash
# cfg5: the priority ladder's band (diag CNMF_ALS_PRIO) on the round-4 product kernel, same box
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
D=gpurun_out/${1:-als_prio2}; mkdir -p $D
B="timeout -k 10 200 python -u bench.py --solver als --steps 200 --warmup 50 --no-cpu"
for r in 1 2; do
  for p in 0 1 2 3 4; do
    CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_diag.so CNMF_ALS_PRIO=$p $B > $D/p${p}_r$r.json 2> $D/p${p}_r$r.err || exit 1
  done
done
echo "exit=0"
