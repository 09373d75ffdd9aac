#!/bin/bash
# the product build: the full GPU suite, smoke, the default bench line and cfg5's
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
D=gpurun_out/${1:-r4g}; mkdir -p $D
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $D/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -u __graft_entry__.py smoke > $D/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $D/bench.json 2> $D/bench.err &&
timeout -k 10 200 python -u bench.py --solver als --steps 200 --warmup 50 --no-cpu > $D/bench_als.json 2> $D/bench_als.err
rc=$?; echo "exit=$rc"; exit $rc
