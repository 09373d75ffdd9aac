#!/bin/bash
# cfg5: per-iteration time vs the launch length and the warmup (is a 200-iteration launch slower?)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
D=gpurun_out/${1:-als_len}; mkdir -p $D
B="timeout -k 10 200 python -u bench.py --solver als --no-cpu"
$B --steps 20 --warmup 0 > $D/s20_w0.json 2> $D/s20_w0.err &&
$B --steps 20 --warmup 200 > $D/s20_w200.json 2> $D/s20_w200.err &&
$B --steps 200 --warmup 0 > $D/s200_w0.json 2> $D/s200_w0.err &&
$B --steps 200 --warmup 50 > $D/s200_w50.json 2> $D/s200_w50.err
rc=$?; echo "exit=$rc"; exit $rc
