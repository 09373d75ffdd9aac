#!/bin/bash
# cfg4 bench with two events around the timed stretch (vs tune()'s per-iteration figure), cfg4 tests
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
D=gpurun_out/${1:-cfg4ev}; mkdir -p $D
B="timeout -k 10 300 python -u bench.py --features 300 --k 16 --dtype bf16 --no-cpu"
$B --steps 100 --warmup 5 > $D/bench_cfg4.json 2> $D/bench_cfg4.err &&
$B --steps 100 --warmup 100 > $D/bench_cfg4_w100.json 2> $D/bench_cfg4_w100.err &&
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_bench_dist.py tests/test_gpu_cfg4_persistent.py > $D/pytest.log 2>&1
rc=$?; echo "exit=$rc"; exit $rc
