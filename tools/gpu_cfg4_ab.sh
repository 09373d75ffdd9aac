#!/bin/bash
# cfg4 A/B on one box: bf16 parity tests on the in-tree library, then the cfg4 bench line alternating
# between the in-tree library and cnmf_amd/libcnmf_hip_prev.so (a build of the previous source),
# then kernel-trace stats of the in-tree library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/${1:-cfg4_ab}
mkdir -p $D
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v -s -p no:cacheprovider --timeout 600 --timeout-method thread"
timeout -k 10 900 $T -m gpu tests/test_gpu_parity.py tests/test_gpu_config_lengths.py -k "bf16 or cfg4 or split" > $D/pytest.log 2>&1 || exit 1
B="bench.py --features 300 --k 16 --dtype bf16 --steps 100 --warmup 5 --no-cpu"
for r in 1 2 3; do
  timeout -k 10 300 python -u $B > $D/new_$r.json 2> $D/new_$r.err || exit 1
  [ -f cnmf_amd/libcnmf_hip_prev.so ] || continue
  CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_prev.so timeout -k 10 300 python -u $B > $D/prev_$r.json 2> $D/prev_$r.err || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o cfg4 --output-format csv -- python3 $B > $D/prof.log 2>&1 || exit 1
echo "exit=0"
