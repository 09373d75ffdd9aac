#!/bin/bash
# Round 4: the new GPU tests first (device tol through the exchange, cfg3 as 8 ranks), then the
# whole GPU suite on the pruned library, then the driver's bench form x2 and the 500-step line.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
D=gpurun_out/${1:-r4a}; mkdir -p $D
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 900 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_sharded_tol.py > $D/pytest_sharded_tol.log 2>&1 &&
timeout -k 10 600 $T -s tests/test_gpu_cfg3_8ranks.py > $D/pytest_cfg3_8ranks.log 2>&1 &&
timeout -k 10 900 $T tests -m gpu --deselect tests/test_gpu_cfg3_8ranks.py --deselect tests/test_gpu_sharded_tol.py > $D/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_df1.json 2> $D/bench_df1.err &&
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $D/bench_df2.json 2> $D/bench_df2.err &&
timeout -k 10 300 python -u bench.py --no-cpu > $D/bench_500.json 2> $D/bench_500.err
echo "exit=$?"
