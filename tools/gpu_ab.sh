#!/bin/bash
# Same-box A/B/... of environment settings: bench.py alternating the arms, 3 rounds each.
#   bash tools/gpu_ab.sh "CNMF_TEAMS=1" "CNMF_TEAMS=2" [-- bench args]
# (an arm is a space-separated list of VAR=value; "X=1" for the defaults)
set -o pipefail
mkdir -p gpurun_out/ab
arms=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do arms+=("$1"); shift; done
[ "$1" = "--" ] && shift
for r in 1 2 3; do
  for i in "${!arms[@]}"; do
    env ${arms[$i]} timeout -k 10 200 python bench.py --no-cpu "$@" > gpurun_out/ab/arm${i}_r$r.log 2>&1 || exit 1
  done
done
python3 - "${arms[@]}" <<'PY'
import json, glob, sys
for i, arm in enumerate(sys.argv[1:]):
    v = []
    for f in sorted(glob.glob(f"gpurun_out/ab/arm{i}_r*.log")):
        for line in open(f):
            if line.startswith("{"):
                v.append(json.loads(line)["roofline"]["avg_us_per_iteration_in_launch"])
    print(f"{arm:60s}", v)
PY
