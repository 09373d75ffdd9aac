"""Diagnostic: the persistent constrained-ALS launch against the per-iteration launches on the same
inputs (W, H relative differences after n iterations, the error word, the Frobenius error)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from cnmf_amd.solver import ALSPlan  # noqa: E402
from cnmf_amd.synthetic import iop_spectra, random_init  # noqa: E402


def run(X, W0, H0, n, persistent, delta, lam):
    plan = ALSPlan(torch.from_numpy(X).cuda(), 4, sum_to_one=delta, smoothness=lam)
    plan.set_W(torch.from_numpy(W0))
    plan.set_H(torch.from_numpy(H0))
    if not persistent:
        plan.persistent = False
    plan.iterate(n)
    torch.cuda.synchronize()
    errw = int(plan.counter[plan.err_word].item())
    return plan.W.cpu().numpy().astype(np.float64), plan.H64.cpu().numpy(), errw, plan.frobenius_error()


def rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


for N in (3008, 40000, 1_000_000):
    X = iop_spectra(N, 81, seed=0, dtype=np.float32)
    W0, H0 = random_init(X, 4, 42)
    for delta, lam in ((0.0, 0.0), (10.0, 1.0)):
        for n in (1, 2, 5):
            Wp, Hp, ep, fp = run(X, W0, H0, n, True, delta, lam)
            Wr, Hr, er, fr = run(X, W0, H0, n, False, delta, lam)
            print(f"N={N} delta={delta} lam={lam} n={n}: relW={rel(Wp, Wr):.2e} relH={rel(Hp, Hr):.2e} "
                  f"err_words={ep},{er} frob={fp:.6g} vs {fr:.6g}", flush=True)
