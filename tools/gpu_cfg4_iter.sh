#!/bin/bash
# cfg4 iteration loop: bf16 parity tests, the ALS H-step tests, and the cfg4 bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/cfg4_iter
mkdir -p $D
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 180 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_parity.py tests/test_gpu_als.py -m gpu -k "bf16 or h_step" > $D/pytest.log 2>&1 &&
timeout -k 10 300 python -u bench.py --features 300 --k 16 --dtype bf16 --steps 100 --warmup 5 --no-cpu > $D/bench_cfg4.json 2> $D/bench_cfg4.err
rc=$?
echo "exit=$rc"
exit $rc
