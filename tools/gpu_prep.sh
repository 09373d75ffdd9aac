#!/bin/bash
# The bench with the prepared (pre-marshalled) library call: driver form and default cfg2, the ALS
# and weighted driver forms, and the one-rank multi-GPU form; persistent GPU tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/prep
mkdir -p $D
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread"
B="timeout -k 10 300 python -u bench.py"
$B --steps 20 --warmup 5 > $D/cfg2_driver.json 2> $D/e1 &&
$B --steps 20 --warmup 5 --no-cpu > $D/cfg2_driver2.json 2> $D/e2 &&
$B --no-cpu > $D/cfg2.json 2> $D/e3 &&
$B --solver als --steps 20 --warmup 5 --no-cpu > $D/als_driver.json 2> $D/e4 &&
$B --weighted --steps 20 --warmup 5 --no-cpu > $D/wmu_driver.json 2> $D/e5 &&
$B --dist --steps 20 --warmup 5 --no-cpu > $D/cfg2_dist_driver.json 2> $D/e6 &&
timeout -k 10 600 $T tests/test_gpu_persistent.py -m gpu > $D/pytest.log 2>&1
rc=$?
echo "exit=$rc"
exit $rc
