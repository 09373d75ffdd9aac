"""The device tolerance test's checked errors against the host loop's on the SAME trajectory
(diagnostic): the closed-form loss of round 5 vs run_mu's per-10-iteration loss
pass (`PASS_LOSS`, the direct residual), both on the product kernel's bit-identical W / H.

    python tools/dbg_tol_cf.py [--n 32000] [--k 4] [--iters 300]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=32000)
    ap.add_argument("--k", type=int, default=4)
    ap.add_argument("--iters", type=int, default=300)
    a = ap.parse_args()
    import torch
    from cnmf_amd.solver import MUPlan
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(a.n, 81, seed=a.n % 97, dtype=np.float32)
    W0, H0 = random_init(X, a.k, 7)

    def plan():
        p = MUPlan(torch.from_numpy(X).cuda(), a.k)
        p.set_W(torch.from_numpy(W0))
        p.set_H(torch.from_numpy(H0))
        return p

    p1 = plan()
    n1, e1 = p1.fit_device_tol(a.iters, 1e-30)
    p2 = plan()
    host = []
    for g in range(0, a.iters, 10):  # the host loop's checks: the direct loss pass every 10 iterations
        host.append((g, p2.frobenius_error()))
        p2.iterate(10)
    torch.cuda.synchronize()
    xsq = float((torch.from_numpy(X).double() ** 2).sum())
    d = dict(e1)
    rows = [{"g": g, "device": d.get(g), "host": h, "rel": (d[g] - h) / h if g in d else None} for g, h in host]
    print(json.dumps({"n_iter": n1, "xsq_host": xsq, "xsq_plan": p1.sumsq_x(),
                      "W_equal": bool(torch.equal(p1.W, p2.W)), "rows": rows}))


if __name__ == "__main__":
    main()
