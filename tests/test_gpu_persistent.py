"""GPU parity of the persistent multi-iteration launch (mu_iter_wt_kernel: fp32, F = 81, k = 4).

The persistent kernel runs the sample pass, the cross-workgroup reduction and the basis update of
every iteration inside ONE launch.  It must give the fp64 oracle's factors within the north_star
bar (1e-5 relative Frobenius) and agree with the per-iteration launch sequence (sample pass +
reduce + basis update) to fp64 summation-order noise.  Shapes are chosen to cover few (4) and many
tiles per workgroup, single and multiple reduction groups, and the regularised update.
"""
import numpy as np
import pytest

from golden_io import rel_fro
from oracle import mu_ref

pytestmark = pytest.mark.gpu

TOL32 = 1e-5


def _plan(X, W0, H0, layout=0, **regs):
    import torch
    from cnmf_amd.solver import MUPlan
    plan = MUPlan(torch.from_numpy(X).cuda(), W0.shape[1], **regs)
    plan.layout = layout
    plan.set_W(torch.from_numpy(W0))
    plan.set_H(torch.from_numpy(H0))
    return plan


def _unfused(plan, n):
    """The per-iteration launch sequence the multi-GPU path uses (no persistent kernel)."""
    from cnmf_amd import _lib
    for _ in range(n):
        plan.sample_pass(_lib.PASS_UPDATE_W | _lib.PASS_ACCUMULATE)
        plan.reduce(plan.n_out, plan.AB)
        plan.basis_update()


@pytest.fixture(params=[4], ids=["wave"])
def layout(request):
    """The persistent launch's layouts in the product library (the plan's `layout` argument): the
    wave tiles.  (The round-1 layouts 1-3 are in the diagnostic build only since round 4.)"""
    return request.param


# 40 / 1000 / 4096 tiles: few tiles per (virtual) workgroup, a padding step for one of the teams
# (odd per-workgroup tile counts), many groups; 15625 = cfg2's tile count
@pytest.mark.parametrize("n_tiles", [40, 1000, 4095, 15625])
def test_persistent_matches_oracle(n_tiles, layout):
    from cnmf_amd.synthetic import iop_spectra, random_init
    N = 64 * n_tiles
    X = iop_spectra(N, 81, seed=n_tiles, dtype=np.float32)
    W0, H0 = random_init(X, 4, 42)
    plan = _plan(X, W0, H0, layout)
    assert plan.persistent, "shape should take the persistent launch"
    n_it = 200 if n_tiles < 15625 else 40  # the full cfg2 size: a shorter oracle run
    plan.iterate(n_it)
    plan.check_sync_error()
    W = plan.W.cpu().numpy()
    H = plan.H64.cpu().numpy()
    Wr, Hr, _ = mu_ref.mu_fit(X.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                              max_iter=n_it, tol=0.0)
    assert rel_fro(W, Wr) <= TOL32 and rel_fro(H, Hr) <= TOL32, (rel_fro(W, Wr), rel_fro(H, Hr))
    # Ht / HHt left behind for the loss pass and the next call are those of the final H
    Ht = plan.Ht.cpu().numpy()
    np.testing.assert_array_equal(Ht[:, :4], H.T)
    np.testing.assert_allclose(plan.HHt.cpu().numpy(), H @ H.T, rtol=1e-12)
    assert plan.counters_at_rest()  # counters back at rest


def test_wave_tiles_are_deterministic_and_the_only_product_layout():
    """Bit-for-bit repeatable, also across split launches; layouts 1-3 are refused by the product."""
    import torch
    from cnmf_amd import _lib
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(64 * 3001, 81, seed=21, dtype=np.float32)
    W0, H0 = random_init(X, 4, 5)
    a, c = _plan(X, W0, H0, 4), _plan(X, W0, H0, 4)
    a.iterate(60)
    for n in (7, 23, 30):
        c.iterate(n)
    a.check_sync_error()
    c.check_sync_error()
    assert torch.equal(a.W, c.W) and torch.equal(a.H64, c.H64)
    assert "wt_kernel" in a.describe()
    with pytest.raises(_lib.HipLibraryError, match="diagnostic"):
        _plan(X, W0, H0, 1).iterate(1)


def test_persistent_agrees_with_per_iteration_launches():
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(64 * 2000, 81, seed=5, dtype=np.float32)
    W0, H0 = random_init(X, 4, 7)
    a = _plan(X, W0, H0)
    b = _plan(X, W0, H0)
    a.iterate(50)
    _unfused(b, 50)
    assert rel_fro(a.W.cpu().numpy(), b.W.cpu().numpy()) < 1e-6
    assert rel_fro(a.H64.cpu().numpy(), b.H64.cpu().numpy()) < 1e-6
    # split launches continue exactly where one launch would be
    c = _plan(X, W0, H0)
    for n in (1, 9, 15, 25):
        c.iterate(n)
    import torch
    assert torch.equal(a.W, c.W) and torch.equal(a.H64, c.H64)


def test_persistent_regularised():
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(64 * 300, 81, seed=9, dtype=np.float32)
    W0, H0 = random_init(X, 4, 3)
    l1W, l2W, l1H, l2H = 0.05, 0.02, 0.1, 0.03
    plan = _plan(X, W0, H0, l1_W=l1W, l2_W=l2W, l1_H=l1H, l2_H=l2H)
    assert plan.persistent
    plan.iterate(100)
    Wr, Hr, _ = mu_ref.mu_fit(X.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                              max_iter=100, tol=0.0, l1_reg_W=l1W, l1_reg_H=l1H, l2_reg_W=l2W,
                              l2_reg_H=l2H)
    W, H = plan.W.cpu().numpy(), plan.H64.cpu().numpy()
    assert rel_fro(W, Wr) <= TOL32 and rel_fro(H, Hr) <= TOL32, (rel_fro(W, Wr), rel_fro(H, Hr))


def test_persistent_tol_stop_through_api():
    """tol > 0: stretches of 10 iterations per launch, the error check between them (SK:872-884)."""
    import cnmf_amd
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(64 * 500, 81, seed=11, dtype=np.float32)
    W0, H0 = random_init(X, 4, 42)
    W, H, n = cnmf_amd.factorise(X, W0.copy(), H0.copy(), n_components=4, init="custom", tol=1e-4,
                                 max_iter=400)
    Wr, Hr, nr = mu_ref.mu_fit(X.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                               max_iter=400, tol=1e-4)
    assert n == nr
    assert rel_fro(W, Wr) <= TOL32 and rel_fro(H, Hr) <= TOL32


def test_failed_persistent_launch_falls_back():
    """a persistent launch that reports a synchronisation failure (forced here
    by a set error word: every waiting workgroup gives up) leaves invalid results; run_mu restores
    the W / H snapshot, re-runs the stretch on the per-iteration path and still matches the oracle."""
    import warnings
    from cnmf_amd.solver import run_mu
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(64 * 1000, 81, seed=31, dtype=np.float32)
    W0, H0 = random_init(X, 4, 8)
    plan = _plan(X, W0, H0)
    assert plan.persistent
    plan.counter[plan.err_word] = 1
    with warnings.catch_warnings(record=True) as rec:
        warnings.simplefilter("always")
        n = run_mu(plan, max_iter=40, tol=0.0)
    assert n == 40 and any("re-run" in str(r.message) for r in rec)
    assert not plan.persistent and plan.counters_at_rest()
    Wr, Hr, _ = mu_ref.mu_fit(X.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                              max_iter=40, tol=0.0)
    W, H = plan.W.cpu().numpy(), plan.H64.cpu().numpy()
    assert rel_fro(W, Wr) <= TOL32 and rel_fro(H, Hr) <= TOL32, (rel_fro(W, Wr), rel_fro(H, Hr))
