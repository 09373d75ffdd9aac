"""CPU ORACLE for the constrained-ALS variant — test infrastructure only.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this module.

The reference (AI-for-Ocean-Science/cnmf v1) ships no solver and sklearn has no constrained ALS, so
this file IS the specification of the variant (DESIGN.md §Constrained ALS); every solve below is
done with `scipy.optimize.nnls` (scipy 1.15, Lawson–Hanson, `scipy/optimize/_nnls.py`) so the GPU
path is checked against an independent exact NNLS solver.  Parity pinning: "parity unpinned" with
respect to the reference (it has no such function); pinned to scipy's NNLS on identical inputs.

One ALS iteration (X: N×F samples-major, W: N×k, H: k×F; fp64):

  W-step (FCLS, per sample i, the HBM pass):
      w_i = argmin_{w >= 0} ||x_i - Hᵀw||² + δ² (1ᵀw - 1)²                       (δ = sum_to_one)
      i.e. NNLS of the augmented system [Hᵀ; δ·1ᵀ] w ≈ [x_i; δ]  (δ = 0: plain NNLS).
  accumulators: A = WᵀX, B = WᵀW  (the new W; the same reductions as the MU path)
  H-step (one Gauss-Seidel sweep over the basis rows j = 0..k-1, rows already updated are used):
      h_j = argmin_{h >= 0} ½ hᵀ(B_jj I + λ L) h - (a_j - Σ_{m≠j} B_jm h_m)ᵀ h      (λ = smoothness)
      with L = DᵀD, D the (F-2)×F second difference ((Dh)_f = h_f - 2h_{f+1} + h_{f+2}).
      This is the exact minimiser of ½||X - WH||² + ½λ||H Dᵀ||²_F over row j with the other rows
      fixed.  A row with B_jj == 0 (an unused component) is left unchanged.
  Stopping: like MU (SK:872-884): with tol > 0 the Frobenius error ||X - WH|| of the current
  factors is checked every 10 iterations (error_at_init from the initial W0, H0) and the loop stops
  when (previous - error) / error_at_init < tol.
"""
from __future__ import annotations

import numpy as np
from scipy.optimize import nnls


def second_difference(F: int) -> np.ndarray:
    D = np.zeros((max(F - 2, 0), F))
    for r in range(F - 2):
        D[r, r:r + 3] = (1.0, -2.0, 1.0)
    return D


def fcls_w(X, H, delta=0.0):
    """Exact per-sample (F)CLS by scipy NNLS on the augmented system."""
    X = np.asarray(X, dtype=np.float64)
    H = np.asarray(H, dtype=np.float64)
    k = H.shape[0]
    A = H.T
    if delta > 0:
        A = np.vstack([A, np.full((1, k), float(delta))])
    W = np.zeros((X.shape[0], k))
    for i in range(X.shape[0]):
        b = X[i] if delta <= 0 else np.append(X[i], float(delta))
        W[i] = nnls(A, b, maxiter=50 * k)[0]
    return W


def fcls_w_enumerate(X, H, delta=0.0):
    """The same minimiser by enumerating passive sets on the Gram form (the GPU's method):
    Q = HHᵀ + δ²11ᵀ, c_i = H x_i + δ²1; for every subset P solve Q_PP w_P = c_P; among the subsets
    with w_P >= 0 take the least objective -½ c_P·w_P (ties: the lowest subset mask)."""
    X = np.asarray(X, dtype=np.float64)
    H = np.asarray(H, dtype=np.float64)
    k = H.shape[0]
    Q = H @ H.T + delta * delta * np.ones((k, k))
    C = X @ H.T + delta * delta
    W = np.zeros((X.shape[0], k))
    best = np.zeros(X.shape[0])
    for mask in range(1, 1 << k):
        P = [j for j in range(k) if mask >> j & 1]
        QP = Q[np.ix_(P, P)]
        if np.linalg.cond(QP) > 1e12:
            continue
        wP = np.linalg.solve(QP, C[:, P].T).T
        f = -0.5 * np.sum(C[:, P] * wP, axis=1)
        ok = np.all(wP >= 0, axis=1) & (f < best)
        W[ok] = 0.0
        W[np.ix_(ok, P)] = wP[ok]
        best[ok] = f[ok]
    return W


def smooth_h_sweep(A, B, H, lam=0.0):
    """One Gauss-Seidel sweep of exact smoothness-penalised NNLS rows (scipy NNLS on the Cholesky
    transform of the row's Gram system: min ||R h - R⁻ᵀ b||², M = RᵀR)."""
    A = np.asarray(A, dtype=np.float64)
    B = np.asarray(B, dtype=np.float64)
    H = np.array(H, dtype=np.float64)
    k, F = H.shape
    L = second_difference(F)
    L = L.T @ L
    for j in range(k):
        if B[j, j] <= 0:
            continue
        b = A[j] - sum(B[j, m] * H[m] for m in range(k) if m != j)
        M = B[j, j] * np.eye(F) + lam * L
        R = np.linalg.cholesky(M).T  # upper: M = RᵀR
        H[j] = nnls(R, np.linalg.solve(R.T, b), maxiter=50 * F)[0]
    return H


def frobenius_error(X, W, H):
    R = np.asarray(X, dtype=np.float64) - np.asarray(W, dtype=np.float64) @ np.asarray(H, dtype=np.float64)
    return float(np.sqrt(np.sum(R * R)))


def als_fit(X, W, H, max_iter=100, tol=0.0, sum_to_one=0.0, smoothness=0.0, return_errors=False,
            w_step="nnls"):
    """The constrained-ALS driver (module docstring).  Returns (W, H, n_iter).  w_step='enumerate'
    solves the W-step with fcls_w_enumerate (the same minimisers as scipy's NNLS — pinned by
    tests/test_als_oracle.py — vectorised over the samples, for oracle runs at 1e5 rows)."""
    w_solve = fcls_w if w_step == "nnls" else fcls_w_enumerate
    X = np.asarray(X, dtype=np.float64)
    W = np.array(W, dtype=np.float64)
    H = np.array(H, dtype=np.float64)
    errors = []
    if tol > 0:
        error_at_init = frobenius_error(X, W, H)
        previous = error_at_init
        errors.append((0, error_at_init))
    it = 0
    for it in range(1, max_iter + 1):
        W = w_solve(X, H, sum_to_one)
        H = smooth_h_sweep(W.T @ X, W.T @ W, H, smoothness)
        if tol > 0 and it % 10 == 0:
            error = frobenius_error(X, W, H)
            errors.append((it, error))
            if (previous - error) / error_at_init < tol:
                break
            previous = error
    if return_errors:
        return W, H, it, errors
    return W, H, it
