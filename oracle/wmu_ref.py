"""CPU ORACLE — test infrastructure only, never shipped as a product path.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this
module, and only as the checker.  The product (`cnmf_amd`) never imports it.

What it restates.  SURVEY.md §8(f) row 2, the weighted / masked multiplicative update, which
neither the reference (its `cnmf/__init__.py` is empty) nor its declared solver dependency
scikit-learn defines.  It is the build's own spec, the standard weighted Frobenius MU (per-element
weights M >= 0; M = 0 marks a missing value, M = 1/σ² an uncertainty weight):

    W <- W o ((M o X) Hᵀ) / ((M o (W H)) Hᵀ)
    H <- H o (Wᵀ (M o X)) / (Wᵀ (M o (W H)))          (with the new W)

in the iteration order of SK:831-870 (W first), zero denominators replaced by float32 eps as
SK:620 / SK:706, and the tol test of SK:872-884 on the weighted error sqrt(Σ m (x − wh)²).
SK = `sklearn/decomposition/_nmf.py` 1.7.2.

Parity pinning.  With M = 1 every formula reduces to SK's unweighted Frobenius MU, so
`tests/test_wmu_oracle.py` checks this module against the sklearn-generated goldens in
`tests/golden/` (M = 1, bit-for-bit in fp64).  Weighted results (M != 1) are "parity unpinned"
with respect to the reference, which has no such function; they are checked for the properties
the spec implies (a zero weight makes an element irrelevant; the weighted error never increases).
"""
from __future__ import annotations

import numpy as np

EPSILON = np.finfo(np.float32).eps  # SK:39


def weighted_error(X, M, W, H):
    """sqrt(Σ m·(x − (WH))²) — SK:85-129's beta=2 error with per-element weights."""
    R = X - W @ H
    return float(np.sqrt(np.sum(M * R * R)))


def update_w(X, M, W, H):
    """W-step (the weighted form of SK:540-554 + SK:620-629)."""
    num = (M * X) @ H.T
    den = (M * (W @ H)) @ H.T
    den[den == 0] = EPSILON
    return W * (num / den)


def update_h(X, M, W, H):
    """H-step with the new W (the weighted form of SK:639-640 + SK:706-726)."""
    num = W.T @ (M * X)
    den = W.T @ (M * (W @ H))
    den[den == 0] = EPSILON
    return H * (num / den)


def wmu_fit(X, M, W, H, max_iter=200, tol=1e-4):
    """The driver of SK:731-893 for the weighted update; returns (W, H, n_iter)."""
    W, H = W.copy(), H.copy()
    error_at_init = previous_error = weighted_error(X, M, W, H) if tol > 0 else None
    n_iter = 0
    for n_iter in range(1, max_iter + 1):
        W = update_w(X, M, W, H)
        H = update_h(X, M, W, H)
        if tol > 0 and n_iter % 10 == 0:
            error = weighted_error(X, M, W, H)
            if (previous_error - error) / error_at_init < tol:
                break
            previous_error = error
    return W, H, n_iter
