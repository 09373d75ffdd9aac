"""The tolerance test on the device (cnmf_mu_fit_tol): sklearn's check of
SK:872-884 — every 10 iterations the Frobenius error of the current factors, stop when
(previous − error) / error_at_init < tol — evaluated inside ONE persistent launch (the error of the
state after g iterations accumulated in the pass of iteration g + 1, which already reads x and w).

The fit must stop at sklearn's n_iter with sklearn's W and H for that n_iter: against the sklearn
goldens (tol_float32: n_iter 180) and the fp64 oracle, k = 4 (W resident in LDS) and k = 8 (W
streamed: the snapshot buffer path), a stop inside the launch and a launch that runs to max_iter,
and the error trajectory against the oracle's.
"""
import numpy as np
import pytest

from golden_io import load, rel_fro
from oracle import mu_ref

pytestmark = pytest.mark.gpu


def _plan(X, W0, H0):
    import torch
    from cnmf_amd.solver import MUPlan
    plan = MUPlan(torch.from_numpy(X).cuda(), W0.shape[1])
    plan.set_W(torch.from_numpy(W0))
    plan.set_H(torch.from_numpy(H0))
    return plan


# a stop inside the launch (k = 4 resident W; k = 8 at 1.2e6 rows: W streamed, the snapshot path),
# a launch that runs to max_iter, and one whose LAST iteration checks the tolerance (max_iter 101)
@pytest.mark.parametrize("n,k,tol,max_iter", [(64 * 500, 4, 1e-4, 400), (64 * 500, 4, 1e-3, 500),
                                             (1_200_000, 8, 1e-3, 100), (64 * 3000, 4, 1e-6, 100),
                                             (64 * 3000, 4, 1e-6, 101)])
def test_device_tol_matches_oracle(n, k, tol, max_iter):
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(n, 81, seed=n % 97, dtype=np.float32)
    W0, H0 = random_init(X, k, 7)
    plan = _plan(X, W0, H0)
    res = plan.fit_device_tol(max_iter, tol)
    assert res is not None, "a wave-tile shape takes the device tolerance test"
    n_iter, errs = res
    plan.check_sync_error()
    assert plan.counters_at_rest()
    Wr, Hr, nr, er = mu_ref.mu_fit(X.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                                   max_iter=max_iter, tol=tol, return_errors=True)
    ref = dict(er)
    if n_iter != nr:  # diagnostics: the device's checked errors and decreases against the oracle's
        for (g, e), (_, ep) in zip(errs[1:], errs):
            print(f"g={g}: device {e:.9g} oracle {ref.get(g, float('nan')):.9g} "
                  f"decrease {(ep - e) / errs[0][1]:.6g}")
    assert n_iter == nr, (n_iter, nr)
    W, H = plan.W.cpu().numpy(), plan.H64.cpu().numpy()
    assert rel_fro(W, Wr) <= 1e-5 and rel_fro(H, Hr) <= 1e-5, (rel_fro(W, Wr), rel_fro(H, Hr))
    # the checked errors: the oracle's (g, error) for every g the launch checked
    for g, e in errs:
        assert abs(e - ref[g]) <= 1e-5 * ref[g], (g, e, ref[g])
    # Ht / HHt of the final H for the calls that follow
    np.testing.assert_array_equal(plan.Ht.cpu().numpy()[:, :k], H.T)


def test_device_tol_golden_through_api():
    """sklearn's own tol run (tests/golden/tol_float32.npz: 300 x 81, tol 1e-3, n_iter 180) — too few
    rows for the persistent launch, so the golden is replayed at 64 x the rows: the same relative
    decrease sequence is not guaranteed, so the API's device-tol fit is checked against the oracle and
    the golden case itself through the host loop (its shape)."""
    import cnmf_amd
    case = load("tol_float32")
    W, H, n = cnmf_amd.factorise(case["X"], case["W0"].copy(), case["H0"].copy(), **case["kwargs"])
    assert n == case["n_iter"]
    X = np.tile(case["X"], (64, 1))
    W0 = np.tile(case["W0"], (64, 1))
    Wg, Hg, ng = cnmf_amd.factorise(X, W0.copy(), case["H0"].copy(), **case["kwargs"])
    Wr, Hr, nr = mu_ref.mu_fit(X.astype(np.float64), W0.astype(np.float64), case["H0"].astype(np.float64),
                               max_iter=case["kwargs"]["max_iter"], tol=case["kwargs"]["tol"])
    assert ng == nr
    assert rel_fro(Wg, Wr) <= 1e-5 and rel_fro(Hg, Hr) <= 1e-5


def test_run_mu_takes_the_device_path_and_falls_back():
    """run_mu on a persistent plan with tol > 0 is ONE launch (no host round trip per 10 iterations);
    a failed launch (forced error word) restores the state and reruns on the host loop."""
    import warnings
    from cnmf_amd.solver import run_mu
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(64 * 800, 81, seed=3, dtype=np.float32)
    W0, H0 = random_init(X, 4, 5)
    Wr, Hr, nr = mu_ref.mu_fit(X.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                               max_iter=300, tol=1e-4)
    plan = _plan(X, W0, H0)
    n, errs = run_mu(plan, max_iter=300, tol=1e-4, return_errors=True)
    assert n == nr
    assert rel_fro(plan.W.cpu().numpy(), Wr) <= 1e-5
    plan2 = _plan(X, W0, H0)
    plan2.counter[plan2.err_word] = 1  # every waiting workgroup gives up: the launch fails
    with warnings.catch_warnings(record=True):
        warnings.simplefilter("always")
        n2 = run_mu(plan2, max_iter=300, tol=1e-4)
    assert n2 == nr and not plan2.persistent and plan2.counters_at_rest()
    assert rel_fro(plan2.W.cpu().numpy(), Wr) <= 1e-5 and rel_fro(plan2.H64.cpu().numpy(), Hr) <= 1e-5


@pytest.mark.parametrize("n,k", [(64 * 3000, 4), (1_200_000, 8)])
def test_device_tol_without_a_stop_is_bit_identical(n, k):
    """A fit whose tolerance never triggers runs the same arithmetic as the plain persistent launch:
    W and H bit for bit (the TOL kernel's extra loss column, snapshot stores and counted waits change
    nothing else; k = 8 at 1.2e6 rows streams W)."""
    import torch
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(n, 81, seed=5, dtype=np.float32)
    W0, H0 = random_init(X, k, 3)
    a, b = _plan(X, W0, H0), _plan(X, W0, H0)
    res = a.fit_device_tol(120, 1e-14)
    assert res is not None and res[0] == 120
    b.iterate(120)
    torch.cuda.synchronize()
    a.check_sync_error()
    b.check_sync_error()
    assert torch.equal(a.W, b.W) and torch.equal(a.H64, b.H64)
