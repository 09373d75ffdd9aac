"""CPU checks of the constrained-ALS oracle (oracle/als_ref.py).

The variant has no reference or sklearn counterpart; these tests pin its two solvers: the per-sample
FCLS (scipy NNLS on the augmented system == the GPU's passive-set enumeration on the Gram form) and
the smoothness-penalised basis rows (scipy NNLS on the Cholesky transform == the KKT conditions).
"""
import numpy as np
import pytest

from oracle import als_ref


def _problem(seed, N=300, F=40, k=4):
    rng = np.random.default_rng(seed)
    H = rng.random((k, F)) + 0.05
    Wt = rng.dirichlet(0.2 * np.ones(k), size=N)  # sparse abundances: active bounds
    X = Wt @ H + 0.02 * rng.standard_normal((N, F))
    return np.clip(X, 0, None), H


@pytest.mark.parametrize("delta", [0.0, 1.0, 10.0])
@pytest.mark.parametrize("k", [1, 2, 3, 4])
def test_fcls_enumeration_matches_scipy_nnls(delta, k):
    X, H = _problem(k, k=k)
    H = H + np.random.default_rng(9).random(H.shape)  # some negative correlations / active bounds
    W1 = als_ref.fcls_w(X, H, delta)
    W2 = als_ref.fcls_w_enumerate(X, H, delta)
    np.testing.assert_allclose(W2, W1, rtol=1e-9, atol=1e-11)
    assert (W1 >= 0).all()
    if k > 1 and delta < 10:
        assert (W1 == 0).any()  # the bound is active somewhere (the test exercises it)


def test_sum_to_one_weight_pulls_rows_to_the_simplex():
    X, H = _problem(3)
    s = [np.abs(als_ref.fcls_w(X, H, d).sum(1) - 1).mean() for d in (0.0, 1.0, 100.0)]
    assert s[2] < s[1] < s[0] and s[2] < 1e-3


@pytest.mark.parametrize("lam", [0.0, 0.5, 20.0])
def test_smooth_row_kkt(lam):
    rng = np.random.default_rng(1)
    X, H = _problem(5)
    W = als_ref.fcls_w(X, H, 1.0)
    A, B = W.T @ X, W.T @ W
    H0 = rng.random(H.shape)
    H1 = als_ref.smooth_h_sweep(A, B, H0, lam)
    F = H.shape[1]
    D = als_ref.second_difference(F)
    L = D.T @ D
    for j in range(H.shape[0]):  # KKT of row j's subproblem with rows < j new and > j old
        Hc = np.vstack([H1[:j + 1], H0[j + 1:]])
        b = A[j] - sum(B[j, m] * Hc[m] for m in range(H.shape[0]) if m != j)
        g = (B[j, j] * np.eye(F) + lam * L) @ H1[j] - b
        h = H1[j]
        scale = np.abs(b).max()
        assert (h >= 0).all()
        assert np.all(g[h > 0] == pytest.approx(0, abs=1e-9 * scale))
        assert (g[h == 0] >= -1e-9 * scale).all()


def test_als_fit_decreases_objective_and_tol_stop():
    X, H = _problem(7, N=200, F=30)
    rng = np.random.default_rng(2)
    H0 = rng.random(H.shape)
    W0 = rng.random((X.shape[0], H.shape[0]))
    _, _, n, errs = als_ref.als_fit(X, W0, H0, max_iter=200, tol=1e-4, sum_to_one=1.0,
                                    smoothness=0.1, return_errors=True)
    e = [v for _, v in errs]
    assert all(b <= a * (1 + 1e-9) for a, b in zip(e[1:], e[2:]))
    assert n < 200 and n % 10 == 0
