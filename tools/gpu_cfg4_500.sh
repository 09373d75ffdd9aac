#!/bin/bash
# cfg4 bench at 100 and 500 timed steps (fixed launch / sync costs amortised), one box
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
D=gpurun_out/${1:-cfg4_500}; mkdir -p $D
B="timeout -k 10 300 python -u bench.py --features 300 --k 16 --dtype bf16 --no-cpu"
$B --steps 100 --warmup 5 > $D/bench_cfg4_100.json 2> $D/bench_cfg4_100.err &&
$B --steps 500 --warmup 20 > $D/bench_cfg4_500.json 2> $D/bench_cfg4_500.err
rc=$?; echo "exit=$rc"; exit $rc
