#!/bin/bash
# Same-box A/B of two builds of the library (tools/ab/libA.so vs libB.so, ABI-compatible):
# alternating bench runs (no CPU baseline), ROUNDS rounds, for each bench argument set in ARGS
# (';'-separated).  Each run under its own time limit; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ab
ROUNDS=${ROUNDS:-2}
IFS=';' read -ra SETS <<< "${ARGS:---steps 500 --warmup 1000}"
n=0
for r in $(seq 1 $ROUNDS); do
  for v in A B; do
    for a in "${SETS[@]}"; do
      n=$((n+1))
      CNMF_HIP_LIB=tools/ab/lib$v.so timeout -k 10 240 python -u bench.py --no-cpu $a > gpurun_out/ab/run${n}_$v.json 2> gpurun_out/ab/run${n}_$v.err || { echo "fail $v $a"; exit 1; }
      python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/run${n}_$v.json')); print('$v', '$a', d['value'], d['roofline']['avg_us_per_iteration_in_launch'], d['roofline']['frac'])"
    done
  done
done
