#!/bin/bash
# One GPU-box session: parity tests, smoke, bench (default and the driver's short form), the two
# HBM-traffic PMC passes (FETCH_SIZE, WRITE_SIZE; each its own run) and the kernel-trace stats of
# the bench.  (Round 1 saw one rocprofv3 abort at process exit after a COOPERATIVE persistent
# launch; persistent launches have been plain launches since, and every profile since finished
# cleanly.)  Each GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread"
P="timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv"
timeout -k 10 900 $T tests -m gpu > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_driver_form.log 2>&1 &&
$P --pmc FETCH_SIZE -d gpurun_out/pmc/fetch -o fetch -- python3 tools/prof_pass.py > gpurun_out/pmc/fetch.log 2>&1 &&
$P --pmc WRITE_SIZE -d gpurun_out/pmc/write -o write -- python3 tools/prof_pass.py > gpurun_out/pmc/write.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 500 --warmup 500 --no-cpu > gpurun_out/prof.log 2>&1
rc=$?
echo "exit=$rc"
exit $rc
