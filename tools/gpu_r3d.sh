#!/bin/bash
# Round 3: new tests, the whole GPU suite, smoke, then the perf probes (tools/gpu_r3c.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/${1:-r3d}
mkdir -p $D
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -s -p no:cacheprovider --timeout 600 --timeout-method thread"
timeout -k 10 900 $T -m gpu tests/test_gpu_device_tol.py tests/test_gpu_mf8.py tests/test_gpu_multidevice.py tests/test_gpu_tall_default.py tests/test_gpu_init.py tests/test_gpu_config_lengths.py tests/test_gpu_bench_dist.py > $D/pytest_new.log 2>&1 &&
timeout -k 10 1200 $T tests -m gpu > $D/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 &&
bash tools/gpu_r3c.sh ${1:-r3d}/perf
rc=$?
echo "exit=$rc"
exit $rc
