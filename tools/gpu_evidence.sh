#!/bin/bash
# Evidence on one MI355X (usage: tools/gpu_evidence.sh <dir under gpurun_out>): the GPU test suite, smoke, the default bench line and the
# driver's short form, HBM-traffic PMC passes and kernel-trace stats of the bench, every BASELINE
# config's bench line, the headline shape at the per-GPU shard sizes of the strong-scaling runs
# (N = 2, 4, 8 of V = 1e6), and kernel-trace stats of the cfg5 ALS bench.  Each GPU step has its
# own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/${1:-evidence}
mkdir -p $D/pmc
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -p no:cacheprovider --timeout 180 --timeout-method thread"
P="timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv"
B="timeout -k 10 300 python -u bench.py"
C4="--rows 1000000 --features 300 --k 16 --dtype bf16 --iters 10"
timeout -k 10 1100 $T tests -m gpu > $D/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 &&
$B > $D/bench.json 2> $D/bench.err &&
$B --steps 20 --warmup 5 > $D/bench_driver_form.json 2> $D/bench_driver_form.err &&
$P --pmc FETCH_SIZE -d $D/pmc/fetch -o fetch -- python3 tools/prof_pass.py > $D/pmc/fetch.log 2>&1 &&
$P --pmc WRITE_SIZE -d $D/pmc/write -o write -- python3 tools/prof_pass.py > $D/pmc/write.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python3 bench.py --steps 500 --warmup 500 --no-cpu > $D/prof.log 2>&1 &&
$B --solver als --steps 200 --warmup 50 --cpu-seconds 10 > $D/bench_cfg5.json 2> $D/bench_cfg5.err &&
$B --features 300 --k 16 --dtype bf16 --steps 100 --warmup 5 --no-cpu > $D/bench_cfg4.json 2> $D/bench_cfg4.err &&
timeout -k 10 400 python -u bench.py --rows 10000000 --k 8 --steps 200 --warmup 200 --no-cpu > $D/bench_cfg3.json 2> $D/bench_cfg3.err &&
$B --rows 1250000 --k 8 --steps 500 --warmup 500 --no-cpu > $D/bench_cfg3shard.json 2> $D/bench_cfg3shard.err &&
$B --tol 1e-4 --steps 500 --warmup 500 --no-cpu > $D/bench_tol.json 2> $D/bench_tol.err &&
$B --weighted --steps 200 --warmup 50 --no-cpu > $D/bench_weighted.json 2> $D/bench_weighted.err &&
$B --rows 499968 --steps 500 --warmup 500 --no-cpu > $D/bench_shard_n2.json 2> $D/bench_shard_n2.err &&
$B --rows 249984 --steps 500 --warmup 500 --no-cpu > $D/bench_shard_n4.json 2> $D/bench_shard_n4.err &&
$B --rows 124992 --steps 500 --warmup 500 --no-cpu > $D/bench_shard_n8.json 2> $D/bench_shard_n8.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_als -o als --output-format csv -- python3 bench.py --solver als --steps 200 --warmup 50 --no-cpu > $D/prof_als.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_cfg4 -o cfg4 --output-format csv -- python3 bench.py --features 300 --k 16 --dtype bf16 --steps 50 --warmup 5 --no-cpu > $D/prof_cfg4.log 2>&1 &&
$P --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT -d $D/pmc/c4a -o c4a -- python3 tools/prof_pass.py $C4 > $D/pmc/c4a.log 2>&1 &&
$P --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU_MFMA_BF16 SQ_INSTS_VALU_MFMA_F64 SQ_WAIT_INST_ANY -d $D/pmc/c4b -o c4b -- python3 tools/prof_pass.py $C4 > $D/pmc/c4b.log 2>&1 &&
$P --pmc FETCH_SIZE -d $D/pmc/c4f -o c4f -- python3 tools/prof_pass.py $C4 > $D/pmc/c4f.log 2>&1 &&
$P --pmc WRITE_SIZE -d $D/pmc/c4w -o c4w -- python3 tools/prof_pass.py $C4 > $D/pmc/c4w.log 2>&1
rc=$?
echo "exit=$rc"
exit $rc
