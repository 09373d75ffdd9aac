#!/bin/bash
# Last check of the round's final build: the whole GPU suite, smoke, and the driver's bench forms.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/last
mkdir -p $D
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests -m gpu > $D/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_driver_form.json 2> $D/e1 &&
timeout -k 10 300 python -u bench.py > $D/bench.json 2> $D/e2 &&
timeout -k 10 300 python -u bench.py --features 300 --k 16 --dtype bf16 --steps 100 --warmup 10 --no-cpu > $D/bench_cfg4.json 2> $D/e3 &&
timeout -k 10 300 python -u bench.py --solver als --steps 200 --warmup 50 --cpu-seconds 10 > $D/bench_cfg5.json 2> $D/e4
rc=$?
echo "exit=$rc"
exit $rc
