"""cfg4 (bf16 X, F = 300, k = 16) as ONE persistent launch (mu_iter_bfw_kernel, layout 6):
the bf16 wave-tile pass with the cross-workgroup reduction (a reduce-scatter between two grid
barriers) and the basis update (SK:634-728, fp64, every workgroup on its own LDS copy) inside the
launch.

Checked against the fp64 oracle on the bf16-rounded X (north-star bar 1e-5) at the config's own
500 iterations, against the per-iteration launches (pass + reduce + update: a different fp64
summation order, so agreement to 1e-6), bit-for-bit across split launches, with l1/l2 terms, on
grids small enough that one workgroup reduces hundreds of columns, with the counters back at rest,
and through run_mu's fallback when a launch reports a synchronisation failure.
"""
import numpy as np
import pytest

from golden_io import rel_fro
from oracle import mu_ref

pytestmark = pytest.mark.gpu


def _data(n, seed):
    import torch
    from cnmf_amd.synthetic import iop_spectra, random_init
    X32 = iop_spectra(n, 300, seed=seed, dtype=np.float32)
    Xb = torch.from_numpy(X32).to(torch.bfloat16)
    Xr = Xb.float().numpy()  # the values bf16 holds: the oracle's input
    W0, H0 = random_init(Xr, 16, 42)
    return Xb, Xr, W0, H0


def _plan(Xb, W0, H0, layout=6, **regs):
    """layout 6: the persistent launch (opt-in; MUPlan.tune() times it against layout 4, the
    per-iteration launches)."""
    import torch
    from cnmf_amd.solver import MUPlan
    plan = MUPlan(Xb.cuda(), 16, **regs)
    assert plan.layouts == (4, 6), plan.layouts
    plan.set_layout(layout)
    plan.set_W(torch.from_numpy(W0))
    plan.set_H(torch.from_numpy(H0))
    return plan


@pytest.mark.timeout(600)
def test_persistent_cfg4_500_iterations_matches_oracle():
    import torch
    Xb, Xr, W0, H0 = _data(64 * 1562, 2)  # 99,968 rows: whole 64-sample tiles
    plan = _plan(Xb, W0, H0)
    assert plan.persistent and "mu_iter_bfw_kernel" in plan.describe(), plan.describe()
    plan.iterate(500)
    torch.cuda.synchronize()
    plan.check_sync_error()
    assert plan.counters_at_rest()
    Wr, Hr, _ = mu_ref.mu_fit(Xr.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                              max_iter=500, tol=0.0)
    W, H = plan.W.cpu().numpy(), plan.H64.cpu().numpy()
    ew, eh = rel_fro(W, Wr), rel_fro(H, Hr)
    print(f"persistent cfg4 99968 x 300, 500 it: rel W {ew:.2e} rel H {eh:.2e}")
    assert ew <= 1e-5 and eh <= 1e-5, (ew, eh)
    # the basis state left for the host: Hᵀ of H, HHᵀ = H Hᵀ
    np.testing.assert_array_equal(plan.Ht.cpu().numpy()[:, :16], H.T)
    np.testing.assert_allclose(plan.HHt.cpu().numpy(), H @ H.T, rtol=1e-12)


# 50 tiles: 7 workgroups, each reducing ~723 of the 5056 columns alone; 200 tiles: 25 workgroups,
# one row chunk per column; 3000 tiles: the row-chunked reduce-scatter of the full-size grid
@pytest.mark.timeout(600)
@pytest.mark.parametrize("n_tiles", [50, 200, 3000])
def test_persistent_agrees_with_launches_and_splits(n_tiles):
    import torch
    Xb, Xr, W0, H0 = _data(64 * n_tiles, n_tiles)
    a, b, c = _plan(Xb, W0, H0), _plan(Xb, W0, H0), _plan(Xb, W0, H0, layout=4)
    assert a.persistent and not c.persistent  # c: the per-iteration launches (pass + reduce + update)
    a.iterate(40)
    for n in (1, 9, 30):
        b.iterate(n)
    c.iterate(40)
    torch.cuda.synchronize()
    for p in (a, b):
        p.check_sync_error()
        assert p.counters_at_rest()
    assert torch.equal(a.W, b.W) and torch.equal(a.H64, b.H64)  # bit for bit across split launches
    assert rel_fro(a.W.cpu().numpy(), c.W.cpu().numpy()) < 1e-6
    assert rel_fro(a.H64.cpu().numpy(), c.H64.cpu().numpy()) < 1e-6
    Wr, Hr, _ = mu_ref.mu_fit(Xr.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                              max_iter=40, tol=0.0)
    assert rel_fro(a.W.cpu().numpy(), Wr) <= 1e-5 and rel_fro(a.H64.cpu().numpy(), Hr) <= 1e-5


@pytest.mark.timeout(600)
def test_persistent_cfg4_regularised():
    import torch
    Xb, Xr, W0, H0 = _data(64 * 700, 9)
    l1W, l2W, l1H, l2H = 0.05, 0.02, 0.1, 0.03
    plan = _plan(Xb, W0, H0, l1_W=l1W, l2_W=l2W, l1_H=l1H, l2_H=l2H)
    assert plan.persistent
    plan.iterate(60)
    torch.cuda.synchronize()
    Wr, Hr, _ = mu_ref.mu_fit(Xr.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                              max_iter=60, tol=0.0, l1_reg_W=l1W, l1_reg_H=l1H, l2_reg_W=l2W, l2_reg_H=l2H)
    W, H = plan.W.cpu().numpy(), plan.H64.cpu().numpy()
    assert rel_fro(W, Wr) <= 1e-5 and rel_fro(H, Hr) <= 1e-5, (rel_fro(W, Wr), rel_fro(H, Hr))


@pytest.mark.timeout(600)
def test_failed_persistent_cfg4_launch_falls_back():
    """A set error word makes every workgroup leave at the first grid barrier (results invalid);
    run_mu restores its snapshot, re-runs the stretch on the per-iteration launches and still
    matches the oracle (and the tolerance test, host-side for this shape, gives sklearn's n_iter)."""
    import warnings
    from cnmf_amd.solver import run_mu
    Xb, Xr, W0, H0 = _data(64 * 300, 31)
    plan = _plan(Xb, W0, H0)
    assert plan.persistent
    plan.counter[plan.err_word] = 1
    with warnings.catch_warnings(record=True) as rec:
        warnings.simplefilter("always")
        n = run_mu(plan, max_iter=30, tol=0.0)
    assert n == 30 and any("re-run" in str(r.message) for r in rec)
    assert not plan.persistent and plan.counters_at_rest()
    Wr, Hr, _ = mu_ref.mu_fit(Xr.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                              max_iter=30, tol=0.0)
    W, H = plan.W.cpu().numpy(), plan.H64.cpu().numpy()
    assert rel_fro(W, Wr) <= 1e-5 and rel_fro(H, Hr) <= 1e-5, (rel_fro(W, Wr), rel_fro(H, Hr))
    plan2 = _plan(Xb, W0, H0)
    n2 = run_mu(plan2, max_iter=300, tol=1e-3)
    assert plan2.persistent
    _, _, nr = mu_ref.mu_fit(Xr.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                             max_iter=300, tol=1e-3)
    assert n2 == nr
