#!/bin/bash
# Same-box A/B: bench with the layout tuning vs without, and the device tolerance test vs tol = 0,
# alternating (box-to-box spread is 2-5 %).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/${1:-ab_tune}
mkdir -p $D
export TMPDIR=/tmp PYTHONUNBUFFERED=1
B="timeout -k 10 240 python -u bench.py --no-cpu"
for r in 1 2 3; do
  $B > $D/tune_$r.json 2> $D/e_tune_$r &&
  $B --no-tune > $D/notune_$r.json 2> $D/e_notune_$r &&
  $B --no-tune --tol 1e-4 > $D/tol_$r.json 2> $D/e_tol_$r || exit 1
done
for f in $D/*.json; do python - "$f" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[1].split('/')[-1], d['value'], d['roofline']['avg_us_per_iteration_in_launch'], d['config'].get('layout_tuning_us_per_iteration'))
PY
done
# cfg3 (k = 8): the matrix-core wave tiles (layout 4) vs the VALU wave tiles (CNMF layout 5 via the
# diagnostic switch), on the 1.25e6-row shard and the whole 1e7 rows
for r in 1 2; do
  $B --rows 1250000 --k 8 --steps 200 --warmup 200 > $D/k8shard_mf_$r.json 2> $D/e_k8m_$r &&
  CNMF_HIP_LIB=$PWD/cnmf_amd/libcnmf_hip_diag.so CNMF_PERSIST_VARIANT=5 $B --rows 1250000 --k 8 --steps 200 --warmup 200 > $D/k8shard_valu_$r.json 2> $D/e_k8v_$r || exit 1
done
$B --rows 10000000 --k 8 --steps 50 --warmup 20 > $D/cfg3_mf.json 2> $D/e_cfg3 || exit 1
for f in $D/k8*.json $D/cfg3*.json; do python - "$f" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[1].split('/')[-1], d['value'], d['roofline']['avg_us_per_iteration_in_launch'], d['roofline']['frac'], d['config']['persistent_layout'][:40])
PY
done
