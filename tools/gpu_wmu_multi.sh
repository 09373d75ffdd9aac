#!/bin/bash
# The weighted MU's multi-GPU launch rehearsed on one GPU (self-exchange, two ranks through IPC),
# then the weighted and ALS bench lines through the multi-GPU launch at one rank.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/wmu_multi
mkdir -p $D
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_wmu.py -m gpu > $D/pytest_wmu.log 2>&1 &&
timeout -k 10 300 python -u bench.py --weighted --dist --steps 200 --warmup 50 --no-cpu > $D/bench_wmu_dist.json 2> $D/bench_wmu_dist.err &&
timeout -k 10 300 python -u bench.py --dist --steps 500 --warmup 500 --no-cpu > $D/bench_cfg2_dist.json 2> $D/bench_cfg2_dist.err
rc=$?
echo "exit=$rc"
exit $rc
