"""Sweep diagnostic-build environment switches over one bench.py shape (GPU box; the diag build
reads CNMF_* switches, the product library ignores them).

    python tools/sweep_env.py --lib cnmf_amd/libcnmf_hip_diag.so --reps 2 \\
        --bench "--rows 124992 --no-cpu --steps 500" \\
        --env "CNMF_WT_PD=3" --env "CNMF_WT_PD=4" --env "CNMF_WT_MAXG=128,CNMF_WT_GROUP=8"

Prints one JSON line per run (the env, us per iteration in the launch, it/s, frac) and a summary
line per env (median over the repetitions); every run alternates through the env list so that
clock drift spreads over all of them.
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "cnmf_amd", "libcnmf_hip_diag.so"))
    ap.add_argument("--bench", required=True)
    ap.add_argument("--env", action="append", default=[])
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    envs = [dict(kv.split("=", 1) for kv in e.split(",") if kv) for e in (a.env or [""])]
    res = {i: [] for i in range(len(envs))}
    for r in range(a.reps):
        for i, e in enumerate(envs):
            env = dict(os.environ, CNMF_HIP_LIB=a.lib, **e)
            p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py")] + a.bench.split(),
                               env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
            if p.returncode != 0:
                print(json.dumps({"env": e, "rep": r, "rc": p.returncode, "err": p.stderr[-800:]}), flush=True)
                sys.exit(1)
            d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
            us = d["roofline"]["avg_us_per_iteration_in_launch"]
            res[i].append(us)
            print(json.dumps({"env": e, "rep": r, "us_per_iteration": us, "value": d["value"],
                              "frac": d["roofline"]["frac"], "layout": d["config"].get("persistent_layout")}),
                  flush=True)
    for i, e in enumerate(envs):
        print(json.dumps({"summary": e, "median_us": statistics.median(res[i]), "all": res[i]}), flush=True)


if __name__ == "__main__":
    main()
