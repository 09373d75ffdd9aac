#!/bin/bash
# One gpurun call, several measured steps, stopping at the first failure (round 5's single driver;
# the per-experiment drivers of earlier rounds are in the git history).
#
#   bash tools/gpu_steps.sh <outdir> "<step>" ["<step>" ...]
#
# Tokens of a step are split on whitespace; a '~' inside a token stands for a space
# (pytest -k "als~or~cfg5").
#
# steps:
#   pytest <tag> <pytest args...>      python -m pytest (thread timeouts) -> <tag>.log
#   bench <tag> <bench.py args...>     one bench line -> <tag>.json / .err
#   benchlib <tag> <lib> <args...>     the same on another library file
#   ab <tag> <n> <bench.py args...>    same-box A/B: tools/ab/libcnmf_hip_base.so (base) and the
#                                      product library alternating n times -> <tag>_{base,prod}_r<i>.json
#   timeline <tag> <args...>           tools/timeline_persist.py on the stamps build -> <tag>.log
#   tlbase <tag> <args...>             the same on tools/ab/libcnmf_hip_base_stamps.so (A/B)
#   tllib <tag> <lib> <args...>        the same on another stamps library file
#   smoke                              __graft_entry__.smoke() -> smoke.log
#   prof <tag> <bench.py args...>      rocprofv3 --kernel-trace --stats of a bench run -> <tag>/
#   pmc <tag> "<counters>" <script args...>  one rocprofv3 --pmc pass over a python script -> <tag>/
#   py <tag> <script args...>          python <script> -> <tag>.log
#   benchenv <tag> <VAR=v> <lib> <bench.py args...>   bench on <lib> with one diagnostic switch set
#   tlenv <tag> <VAR=v> <args...>      the timeline on the stamps build with one diagnostic switch set
#   pytestenv <tag> <VAR=v> <lib> <pytest args...>     pytest on <lib> with one diagnostic switch set
#   pylib <tag> <lib> <script args...> the same with CNMF_HIP_LIB=<lib>
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
D=gpurun_out/$1; shift; mkdir -p "$D"
BASE=${AB_BASE:-tools/ab/libcnmf_hip_base.so}
for st in "$@"; do
  set -- $st
  kind=$1; tag=$2; shift 2
  args=(); for a in "$@"; do args+=("${a//\~/ }"); done; set -- "${args[@]}"  # '~' in a token = a space
  echo "[steps] $kind $tag $* ($(date +%T))"
  case $kind in
    pytest)
      timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread "$@" > "$D/$tag.log" 2>&1 || { tail -30 "$D/$tag.log"; exit 1; } ;;
    bench)
      timeout -k 10 400 python -u bench.py "$@" > "$D/$tag.json" 2> "$D/$tag.err" || { tail -20 "$D/$tag.err"; exit 1; } ;;
    benchlib)  # one bench line on another library: benchlib <tag> <lib> <bench args>
      lib=$1; shift
      CNMF_HIP_LIB=$lib timeout -k 10 400 python -u bench.py "$@" > "$D/$tag.json" 2> "$D/$tag.err" || { tail -20 "$D/$tag.err"; exit 1; } ;;
    ab)
      n=$1; shift
      for r in $(seq 1 "$n"); do
        CNMF_HIP_LIB=$BASE timeout -k 10 300 python -u bench.py "$@" > "$D/${tag}_base_r$r.json" 2> "$D/${tag}_base_r$r.err" || { tail -20 "$D/${tag}_base_r$r.err"; exit 1; }
        timeout -k 10 300 python -u bench.py "$@" > "$D/${tag}_prod_r$r.json" 2> "$D/${tag}_prod_r$r.err" || { tail -20 "$D/${tag}_prod_r$r.err"; exit 1; }
      done ;;
    tlbase)  # the timeline on the base library's stamps build (same-box A/B of the timeline)
      CNMF_HIP_LIB=tools/ab/libcnmf_hip_base_stamps.so timeout -k 10 300 python -u tools/timeline_persist.py "$@" > "$D/$tag.log" 2>&1 || { tail -20 "$D/$tag.log"; exit 1; } ;;
    tllib)
      lib=$1; shift
      CNMF_HIP_LIB=$lib timeout -k 10 300 python -u tools/timeline_persist.py "$@" > "$D/$tag.log" 2>&1 || { tail -20 "$D/$tag.log"; exit 1; } ;;
    timeline)
      CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_stamps.so timeout -k 10 300 python -u tools/timeline_persist.py "$@" > "$D/$tag.log" 2>&1 || { tail -20 "$D/$tag.log"; exit 1; } ;;
    smoke)
      timeout -k 10 200 python -u __graft_entry__.py smoke > "$D/smoke.log" 2>&1 || { tail -20 "$D/smoke.log"; exit 1; } ;;
    prof)
      mkdir -p "$D/$tag"
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$D/$tag" -o run -- python3 -u bench.py "$@" > "$D/$tag/bench.json" 2> "$D/$tag/bench.err" || { tail -20 "$D/$tag/bench.err"; exit 1; } ;;
    pmc)
      ctrs=${1//,/ }; shift
      mkdir -p "$D/$tag"
      timeout -s KILL 120 rocprofv3 --pmc $ctrs -d "$D/$tag" -o run -- python3 -u "$@" > "$D/$tag/out.log" 2>&1 || { tail -20 "$D/$tag/out.log"; exit 1; } ;;
    pylib)
      lib=$1; shift
      CNMF_HIP_LIB=$lib timeout -k 10 400 python -u "$@" > "$D/$tag.log" 2>&1 || { tail -20 "$D/$tag.log"; exit 1; } ;;
    py)
      timeout -k 10 400 python -u "$@" > "$D/$tag.log" 2>&1 || { tail -20 "$D/$tag.log"; exit 1; } ;;
    benchenv)
      kv=$1; lib=$2; shift 2
      env "$kv" CNMF_HIP_LIB=$lib timeout -k 10 400 python -u bench.py "$@" > "$D/$tag.json" 2> "$D/$tag.err" || { tail -20 "$D/$tag.err"; exit 1; } ;;
    tlenv)
      kv=$1; shift
      env "$kv" CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_stamps.so timeout -k 10 300 python -u tools/timeline_persist.py "$@" > "$D/$tag.log" 2>&1 || { tail -20 "$D/$tag.log"; exit 1; } ;;
    pytestenv)
      kv=$1; lib=$2; shift 2
      env "$kv" CNMF_HIP_LIB=$lib timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread "$@" > "$D/$tag.log" 2>&1 || { tail -30 "$D/$tag.log"; exit 1; } ;;
    *) echo "unknown step $kind"; exit 2 ;;
  esac
done
echo "[steps] done ($(date +%T))"
