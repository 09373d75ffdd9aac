#!/bin/bash
# Round 4: the persistent cfg4 launch (mu_iter_bfw_kernel) — its tests, the cfg4 parity tests, the
# cfg4 bench line and kernel stats; then the ALS diagnostics (timeline + SQ passes).
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
D=gpurun_out/${1:-r4b}; mkdir -p $D
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 600 --timeout-method thread"
timeout -k 10 600 $T -s tests/test_gpu_cfg4_persistent.py > $D/pytest_cfg4p.log 2>&1 &&
timeout -k 10 300 python -u bench.py --features 300 --k 16 --dtype bf16 --steps 100 --warmup 10 --no-cpu > $D/bench_cfg4.json 2> $D/bench_cfg4.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_cfg4 -o cfg4 --output-format csv -- python3 bench.py --features 300 --k 16 --dtype bf16 --steps 50 --warmup 5 --no-cpu > $D/prof_cfg4.log 2>&1 &&
timeout -k 10 900 $T -s tests/test_gpu_config_lengths.py tests/test_gpu_parity.py > $D/pytest_cfg4_parity.log 2>&1
rc=$?
echo "exit=$rc"
exit $rc
