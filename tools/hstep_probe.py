"""Time the constrained ALS's H-step on its own (cnmf_als_basis_update = als_basis_kernel: the
Gauss-Seidel sweep of NNLS rows, Hᵀ / HHᵀ and the W-step's passive-set table) at cfg5's regime:
accumulators of 1e6 samples (B_jj large: the Jacobi rows), lambda = 0.5, delta = 1 (diagnostic).

    python tools/hstep_probe.py [--calls 2000] [--lam 0.5]

Prints µs per call (HIP events around `calls` back-to-back launches); with CNMF_HIP_LIB pointing at
a -DCNMF_ALS_NOHSTEP build the difference is the rows' share.
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=2000)
    ap.add_argument("--lam", type=float, default=0.5)
    a = ap.parse_args()
    import torch
    from cnmf_amd.solver import ALSPlan
    from cnmf_amd.synthetic import iop_spectra, random_init
    from oracle import als_ref  # test infrastructure: the accumulators of a realistic state
    Xf = iop_spectra(1_000_000, 81, seed=0, dtype=np.float32)
    X = Xf[:20000].astype(np.float64)
    W0, H0 = random_init(Xf, 4, 42)
    H = H0.astype(np.float64)
    for _ in range(5):  # a few host ALS steps toward cfg5's operating point
        W = als_ref.fcls_w_enumerate(X, H, 1.0)
        s = 1e6 / X.shape[0]
        H = als_ref.smooth_h_sweep(s * (W.T @ X), s * (W.T @ W), H, a.lam)
    W = als_ref.fcls_w_enumerate(X, H, 1.0)
    s = 1e6 / X.shape[0]
    A, B = s * (W.T @ X), s * (W.T @ W)
    plan = ALSPlan(torch.from_numpy(Xf[:20000].copy()).cuda(), 4, sum_to_one=1.0, smoothness=a.lam)
    ab = torch.from_numpy(np.concatenate([A, B], axis=1).ravel()).cuda()
    h0 = torch.from_numpy(H).cuda()
    st = torch.cuda.current_stream()
    res = {}
    for rep in range(3):
        plan.set_H(h0)
        plan.AB.copy_(ab)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(a.calls):  # the same inputs every call (H64 is re-set only per rep: the rows warm-start)
            plan.h_step()
        e1.record(st)
        torch.cuda.synchronize()
        res[rep] = e0.elapsed_time(e1) * 1e3 / a.calls
    print(json.dumps({"lib": os.environ.get("CNMF_HIP_LIB", "product"), "us_per_call": res,
                      "rho_rows": [10 * a.lam / float(B[j, j]) for j in range(4)]}))


if __name__ == "__main__":
    main()
