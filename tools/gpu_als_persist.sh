#!/bin/bash
# cfg5 constrained ALS: GPU parity tests (per-iteration and persistent launches), then the cfg5
# bench line persistent and per-iteration (CNMF_ALS_PERSIST=0), then kernel-trace stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/als
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 180 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_als.py -m gpu > gpurun_out/als/pytest.log 2>&1 &&
timeout -k 10 300 python -u bench.py --solver als --steps 200 --warmup 50 > gpurun_out/als/bench_persistent.json 2> gpurun_out/als/bench_persistent.err &&
CNMF_ALS_PERSIST=0 timeout -k 10 300 python -u bench.py --solver als --steps 100 --warmup 20 --no-cpu > gpurun_out/als/bench_per_iteration.json 2> gpurun_out/als/bench_per_iteration.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/als/prof -o als -- python3 bench.py --solver als --steps 200 --warmup 50 --no-cpu > gpurun_out/als/prof.log 2>&1
echo "rc=$?"
