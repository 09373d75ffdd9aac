#!/bin/bash
# cfg5: the wave H-step's phases (stamps build), then the issue-priority ladder (diag CNMF_ALS_PRIO =
# steps per band) A/B against the product kernel, two rounds, and the ladder's parity.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
D=gpurun_out/${1:-als_prio}; mkdir -p $D
CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_stamps.so timeout -k 10 200 python tools/timeline_persist.py --solver als > $D/timeline.log 2>&1 || exit 1
B="timeout -k 10 200 python -u bench.py --solver als --steps 200 --warmup 50 --no-cpu"
for r in 1 2; do
  $B > $D/als_p0_r$r.json 2> $D/als_p0_r$r.err || exit 1
  for p in 2 4 6; do
    CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_diag.so CNMF_ALS_PRIO=$p $B > $D/als_p${p}_r$r.json 2> $D/als_p${p}_r$r.err || exit 1
  done
done
CNMF_ALS_PRIO=4 CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_stamps.so timeout -k 10 200 python tools/timeline_persist.py --solver als > $D/timeline_p4.log 2>&1 &&
CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_diag.so CNMF_ALS_PRIO=4 timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_als.py > $D/pytest_als_p4.log 2>&1
rc=$?
echo "exit=$rc"
exit $rc
