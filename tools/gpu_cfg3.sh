#!/bin/bash
# cfg2 default bench line, cfg3 (1e7 x 81, k = 8) at one GPU and one cfg3 shard (1.25e6 rows),
# plus the kernel-trace summary of the cfg3 run.  Each GPU step under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/cfg3
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > gpurun_out/cfg3/bench_cfg2.json 2> gpurun_out/cfg3/bench_cfg2.err &&
timeout -k 10 400 python -u bench.py --rows 10000000 --k 8 --steps 200 --warmup 200 --no-cpu > gpurun_out/cfg3/bench_cfg3.json 2> gpurun_out/cfg3/bench_cfg3.err &&
timeout -k 10 300 python -u bench.py --rows 1250000 --k 8 --steps 500 --warmup 500 --no-cpu > gpurun_out/cfg3/bench_cfg3shard.json 2> gpurun_out/cfg3/bench_cfg3shard.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/cfg3/prof -o cfg3 -- python3 bench.py --rows 10000000 --k 8 --steps 100 --warmup 100 --no-cpu --no-tune > gpurun_out/cfg3/prof.log 2>&1
echo "rc=$?"
