#!/bin/bash
# Round 3 perf probes: default bench, device-tol bench, strong-scaling shard sizes, prefetch depth
# (diagnostic build) at the shard sizes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/${1:-r3c}
mkdir -p $D
export TMPDIR=/tmp PYTHONUNBUFFERED=1
B="timeout -k 10 240 python -u bench.py --no-cpu"
$B > $D/bench.json 2> $D/e0 &&
$B --tol 1e-4 --steps 500 --no-tune > $D/bench_tol.json 2> $D/e1 &&
$B --no-tune --steps 500 > $D/bench_notol_notune.json 2> $D/e2 &&
for r in 499968 249984 124992; do
  $B --rows $r --steps 500 --warmup 500 > $D/bench_shard_$r.json 2> $D/es_$r || exit 1
  for pd in 2 4; do
    CNMF_HIP_LIB=$PWD/cnmf_amd/libcnmf_hip_diag.so CNMF_WT_PD=$pd $B --rows $r --steps 500 --warmup 500 --no-tune > $D/bench_shard_${r}_pd$pd.json 2> $D/es_${r}_$pd || exit 1
  done
done
rc=$?
echo "exit=$rc"
exit $rc
