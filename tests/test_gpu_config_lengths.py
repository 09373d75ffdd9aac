"""Parity at the BASELINE configs' own iteration counts.

* cfg4 (bf16 X, F = 300, k = 16, 500 MU iterations): the GPU path against the fp64 oracle run on
  the bf16-rounded X at 1e5 rows (the oracle finishes in seconds there), bar 1e-5; and the full
  1e6 x 300 shape through size-independent properties: bit-identical repeat runs, non-negative
  factors, a monotonically decreasing objective.
* cfg5 (constrained ALS, δ = 1, λ = 0.5, k = 4, 100 iterations) at 1e5 rows against the ALS oracle
  (its W-step by the vectorised passive-set enumeration, pinned to scipy's NNLS by
  tests/test_als_oracle.py), bar 1e-5.
"""
import numpy as np
import pytest

from golden_io import rel_fro
from oracle import mu_ref

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(600)
def test_cfg4_500_iterations_matches_oracle():
    import torch
    import cnmf_amd
    from cnmf_amd.synthetic import iop_spectra, random_init
    X32 = iop_spectra(100_000, 300, seed=2, dtype=np.float32)
    Xb = torch.from_numpy(X32).to(torch.bfloat16)
    Xr = Xb.float().numpy()  # the values bf16 holds
    W0, H0 = random_init(Xr, 16, 42)
    W, H, n = cnmf_amd.factorise(Xb.cuda(), torch.from_numpy(W0).cuda(), torch.from_numpy(H0).cuda(),
                                 n_components=16, init="custom", tol=0.0, max_iter=500)
    assert n == 500
    Wr, Hr, _ = mu_ref.mu_fit(Xr.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                              max_iter=500, tol=0.0)
    ew, eh = rel_fro(W.cpu().numpy(), Wr), rel_fro(H.cpu().numpy(), Hr)
    print(f"cfg4 1e5 x 300 k16 bf16, 500 it: rel W {ew:.2e} rel H {eh:.2e}")
    assert ew <= 1e-5 and eh <= 1e-5, (ew, eh)


@pytest.mark.timeout(600)
def test_cfg4_full_size_matches_oracle():
    """cfg4 at its full 1e6 x 300 (k = 16): the wave-tile pass's fp32 MFMA accumulators chain over
    every tile of a wave (≈ 61 per iteration), so the 1e6-row shape is checked against the fp64
    oracle on the bf16-rounded X too (20 iterations: the oracle's cost), bar 1e-5."""
    import torch
    from cnmf_amd.solver import MUPlan
    from cnmf_amd.synthetic import iop_spectra, random_init
    X32 = iop_spectra(1_000_000, 300, seed=4, dtype=np.float32)
    Xb = torch.from_numpy(X32).to(torch.bfloat16)
    del X32
    Xr = Xb.float().numpy()
    W0, H0 = random_init(Xr, 16, 42)
    plan = MUPlan(Xb.cuda(), 16)
    plan.set_W(torch.from_numpy(W0))
    plan.set_H(torch.from_numpy(H0))
    plan.iterate(20)
    torch.cuda.synchronize()
    W, H = plan.W.cpu().numpy(), plan.H64.cpu().numpy()
    Wr, Hr, _ = mu_ref.mu_fit(Xr.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                              max_iter=20, tol=0.0)
    ew, eh = rel_fro(W, Wr), rel_fro(H, Hr)
    print(f"cfg4 1e6 x 300 k16 bf16, 20 it: rel W {ew:.2e} rel H {eh:.2e}")
    assert ew <= 1e-5 and eh <= 1e-5, (ew, eh)


@pytest.mark.timeout(600)
def test_cfg4_full_size_properties():
    import torch
    from cnmf_amd.solver import MUPlan
    from cnmf_amd.synthetic import iop_spectra, random_init
    X32 = iop_spectra(1_000_000, 300, seed=0, dtype=np.float32)
    W0, H0 = random_init(X32, 16, 42)
    Xb = torch.from_numpy(X32).to(torch.bfloat16).cuda()
    del X32
    outs, errs = [], []
    for rep in range(2):
        plan = MUPlan(Xb, 16)
        plan.set_W(torch.from_numpy(W0))
        plan.set_H(torch.from_numpy(H0))
        e = [plan.frobenius_error()]
        for stretch in (10, 40, 150, 300):  # 500 iterations in all
            plan.iterate(stretch)
            e.append(plan.frobenius_error())
        errs.append(e)
        outs.append((plan.W.clone(), plan.H64.clone()))
        del plan
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert errs[0] == errs[1]
    assert all(b < a for a, b in zip(errs[0], errs[0][1:])), errs[0]
    assert bool((outs[0][0] >= 0).all()) and bool((outs[0][1] >= 0).all())
    print(f"cfg4 full size: errors {errs[0]}")


@pytest.mark.timeout(600)
def test_cfg5_100_iterations_matches_oracle():
    import cnmf_amd
    from oracle import als_ref
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(100_000, 81, seed=5, dtype=np.float32)
    W0, H0 = random_init(X, 4, 42)
    W, H, n = cnmf_amd.factorise(X, W0.copy(), H0.copy(), n_components=4, init="custom", solver="als",
                                 sum_to_one=1.0, smoothness=0.5, tol=0.0, max_iter=100)
    assert n == 100
    Wr, Hr, _ = als_ref.als_fit(X.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                                max_iter=100, tol=0.0, sum_to_one=1.0, smoothness=0.5, w_step="enumerate")
    ew, eh = rel_fro(W, Wr), rel_fro(H, Hr)
    print(f"cfg5 1e5 x 81 k4 ALS, 100 it: rel W {ew:.2e} rel H {eh:.2e}")
    assert ew <= 1e-5 and eh <= 1e-5, (ew, eh)
