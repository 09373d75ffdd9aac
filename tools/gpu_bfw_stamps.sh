#!/bin/bash
# Per-phase cycles of the wave-tile bf16 pass (stamps build), the cfg4 bench line, its parity tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/${1:-bfw_stamps}
mkdir -p $D
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -s -p no:cacheprovider --timeout 600 --timeout-method thread"
timeout -k 10 900 $T -m gpu tests/test_gpu_parity.py tests/test_gpu_config_lengths.py -k "bf16 or cfg4 or split" > $D/pytest_bf16.log 2>&1 || exit 1
CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_stamps.so timeout -k 10 200 python -u tools/stamps_bf16.py > $D/stamps.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --features 300 --k 16 --dtype bf16 --steps 100 --warmup 5 --no-cpu > $D/bench_cfg4.json 2> $D/bench_cfg4.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o cfg4 --output-format csv -- python3 bench.py --features 300 --k 16 --dtype bf16 --steps 50 --warmup 5 --no-cpu > $D/prof.log 2>&1 || exit 1
echo "exit=0"
