#!/bin/bash
# Round 3 check: the new N = 2 bench tests first, then the whole GPU suite, smoke and the driver's
# bench forms.  Usage: tools/gpu_r3.sh <out-subdir> [pytest -k expression]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/${1:-r3}
mkdir -p $D
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_bench_dist.py -m gpu > $D/pytest_bench_dist.log 2>&1 &&
timeout -k 10 900 $T tests -m gpu ${2:+-k "$2"} > $D/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_driver_form.json 2> $D/e1 &&
timeout -k 10 300 python -u bench.py > $D/bench.json 2> $D/e2
rc=$?
echo "exit=$rc"
exit $rc
