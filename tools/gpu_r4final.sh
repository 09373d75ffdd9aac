#!/bin/bash
# Round-4 evidence on one MI355X.  usage: tools/gpu_r4final.sh <dir> <part: 1|2>
#   1: the GPU suite, smoke, the default bench line, the driver's short form, the 500-step line,
#      HBM-traffic PMC passes of cfg2's launch and the kernel-trace stats of the 500-step bench
#   2: every other config's bench line (cfg5 plain / tol, cfg4, cfg3 at full size and its per-GPU
#      shard, cfg2 tol, weighted, the strong-scaling shard sizes) and kernel-trace stats of cfg5 / cfg4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/${1:-r4final}
mkdir -p $D/pmc
export TMPDIR=/tmp PYTHONUNBUFFERED=1
P="timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv"
B="timeout -k 10 300 python -u bench.py"
if [ "${2:-1}" = "1" ]; then
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $D/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 &&
$B > $D/bench.json 2> $D/bench.err &&
$B --steps 20 --warmup 5 > $D/bench_driver_form.json 2> $D/bench_driver_form.err &&
$B --steps 500 --warmup 500 --no-cpu > $D/bench_500.json 2> $D/bench_500.err &&
$P --pmc FETCH_SIZE -d $D/pmc/fetch -o fetch -- python3 tools/prof_pass.py > $D/pmc/fetch.log 2>&1 &&
$P --pmc WRITE_SIZE -d $D/pmc/write -o write -- python3 tools/prof_pass.py > $D/pmc/write.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python3 bench.py --steps 500 --warmup 500 --no-cpu > $D/prof.log 2>&1
else
$B --solver als --steps 200 --warmup 50 --cpu-seconds 10 > $D/bench_cfg5.json 2> $D/bench_cfg5.err &&
$B --solver als --tol 1e-4 --steps 200 --warmup 50 --no-cpu > $D/bench_cfg5_tol.json 2> $D/bench_cfg5_tol.err &&
$B --features 300 --k 16 --dtype bf16 --steps 100 --warmup 5 --no-cpu > $D/bench_cfg4.json 2> $D/bench_cfg4.err &&
timeout -k 10 400 python -u bench.py --rows 10000000 --k 8 --steps 200 --warmup 200 --no-cpu > $D/bench_cfg3.json 2> $D/bench_cfg3.err &&
$B --rows 1250000 --k 8 --steps 500 --warmup 500 --no-cpu > $D/bench_cfg3shard.json 2> $D/bench_cfg3shard.err &&
$B --tol 1e-4 --steps 500 --warmup 500 --no-cpu > $D/bench_tol.json 2> $D/bench_tol.err &&
$B --weighted --steps 200 --warmup 50 --no-cpu > $D/bench_weighted.json 2> $D/bench_weighted.err &&
$B --rows 124992 --steps 500 --warmup 500 --no-cpu > $D/bench_shard_n8.json 2> $D/bench_shard_n8.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_als -o als --output-format csv -- python3 bench.py --solver als --steps 200 --warmup 50 --no-cpu > $D/prof_als.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_cfg4 -o cfg4 --output-format csv -- python3 bench.py --features 300 --k 16 --dtype bf16 --steps 50 --warmup 5 --no-cpu > $D/prof_cfg4.log 2>&1
fi
rc=$?
echo "exit=$rc"
exit $rc
