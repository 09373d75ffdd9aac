#!/bin/bash
# cfg4 persistent after batching its sc1 loads: bench line + end-of-iteration stamps; then the ALS A/B.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
D=gpurun_out/${1:-r4c}; mkdir -p $D
timeout -k 10 300 python -u bench.py --features 300 --k 16 --dtype bf16 --steps 100 --warmup 10 --no-cpu > $D/bench_cfg4.json 2> $D/bench_cfg4.err &&
CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_stamps.so timeout -k 10 200 python -u tools/stamps_bfw_persist.py > $D/stamps_bfw_persist.log 2>&1 &&
bash tools/gpu_als_ab.sh ${1:-r4c}/als_ab
echo "exit=$?"
