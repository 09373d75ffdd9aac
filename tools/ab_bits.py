"""Bit-compare two library builds on the same persistent ALS / MU fit (diagnostic): each run in its
own process with CNMF_HIP_LIB, W and H saved, then compared for exact equality.

    python tools/ab_bits.py --lib-a tools/ab/libcnmf_hip_base.so --lib-b cnmf_amd/libcnmf_hip.so \\
        [--solver als] [--rows 40000] [--iters 20]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_one(a, out):
    sys.path.insert(0, ROOT)
    import torch
    from cnmf_amd.solver import ALSPlan, MUPlan
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(a.rows, 81, seed=3, dtype=np.float32)
    W0, H0 = random_init(X, a.k, 42)
    if a.solver == "als":
        plan = ALSPlan(torch.from_numpy(X).cuda(), a.k, sum_to_one=1.0, smoothness=0.5)
    else:
        plan = MUPlan(torch.from_numpy(X).cuda(), a.k)
    plan.set_W(torch.from_numpy(W0))
    plan.set_H(torch.from_numpy(H0))
    plan.iterate(a.iters)
    torch.cuda.synchronize()
    np.savez(out, W=plan.W.cpu().numpy(), H=plan.H64.cpu().numpy())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib-a", required=True)
    ap.add_argument("--lib-b", required=True)
    ap.add_argument("--solver", default="als", choices=["als", "mu"])
    ap.add_argument("--rows", type=int, default=40000)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--k", type=int, default=4)
    ap.add_argument("--_out", default=None)
    a = ap.parse_args()
    if a._out:
        run_one(a, a._out)
        return
    res = {}
    with tempfile.TemporaryDirectory() as td:
        for tag, lib in (("a", a.lib_a), ("b", a.lib_b)):
            out = os.path.join(td, tag + ".npz")
            cmd = [sys.executable, os.path.abspath(__file__), "--lib-a", a.lib_a, "--lib-b", a.lib_b, "--solver",
                   a.solver, "--rows", str(a.rows), "--iters", str(a.iters), "--k", str(a.k), "--_out", out]
            subprocess.run(cmd, check=True, env=dict(os.environ, CNMF_HIP_LIB=lib), timeout=300)
            res[tag] = np.load(out)
        W_eq = bool(np.array_equal(res["a"]["W"], res["b"]["W"]))
        H_eq = bool(np.array_equal(res["a"]["H"], res["b"]["H"]))
        dW = float(np.abs(res["a"]["W"] - res["b"]["W"]).max())
        dH = float(np.abs(res["a"]["H"] - res["b"]["H"]).max())
    print(json.dumps({"solver": a.solver, "k": a.k, "rows": a.rows, "iters": a.iters, "W_bit_equal": W_eq, "H_bit_equal": H_eq,
                      "max_abs_dW": dW, "max_abs_dH": dH}))
    sys.exit(0 if (W_eq and H_eq) else 4)


if __name__ == "__main__":
    main()
