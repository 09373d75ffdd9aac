#!/bin/bash
# cfg4's persistent launch as opt-in layout 6: its parity tests, the cfg4 bench with tune() choosing
# between layouts 4 and 6, the default bench line and smoke().
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
D=gpurun_out/${1:-r4e}; mkdir -p $D
T="timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
$T tests/test_gpu_cfg4_persistent.py tests/test_gpu_config_lengths.py > $D/pytest_cfg4p.log 2>&1 &&
timeout -k 10 300 python -u bench.py --features 300 --k 16 --dtype bf16 --steps 100 --warmup 10 --no-cpu > $D/bench_cfg4.json 2> $D/bench_cfg4.err &&
timeout -k 10 300 python -u bench.py --features 300 --k 16 --dtype bf16 --steps 100 --warmup 10 --no-cpu --layout 6 > $D/bench_cfg4_l6.json 2> $D/bench_cfg4_l6.err &&
timeout -k 10 120 python -u __graft_entry__.py smoke > $D/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $D/bench.json 2> $D/bench.err
rc=$?
echo "exit=$rc"
exit $rc
