"""CPU ORACLE — test infrastructure only, never shipped as a product path.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this
module, and only as the checker / the timed CPU baseline.  The product (`cnmf_amd`) never imports
it and fails loudly if its HIP library is missing.

What it restates.  The reference (`/root/reference`, AI-for-Ocean-Science/cnmf v1) contains no
solver: `cnmf/__init__.py` is 0 bytes.  The algorithm its declared dependency
scikit-learn (`/root/reference/setup.py:26,30`, unpinned; 1.7.2 in this image) implements for
`solver='mu', beta_loss='frobenius'` is restated here in NumPy, op for op, so that the fp64 result
is bit-identical to sklearn's and the fp32 result follows the same fp32 NumPy arithmetic.
Citations use `SK:` = `sklearn/decomposition/_nmf.py` (1.7.2).

Parity pinning.  `tests/golden/make_golden.py` runs sklearn 1.7.2 itself in the build container and
commits input/output vectors to `tests/golden/*.npz`; `tests/test_oracle.py` checks this module
against every one of them (fp64 bit-exact).  The reference has no tests or fixtures of its own.

Row (a7) — the constrained-ALS variant — has no sklearn counterpart; `fcls_sample` /
`smooth_basis_nnls` below are the build's own spec (DESIGN.md §Constrained ALS), checked against
`scipy.optimize.nnls`.
"""
from __future__ import annotations

import numpy as np

EPSILON = np.finfo(np.float32).eps  # SK:39 — used for fp32 AND fp64 inputs


# --------------------------------------------------------------------------------------------
# a3: loss
# --------------------------------------------------------------------------------------------
def frobenius_error(X, W, H):
    """`_beta_divergence(X, W, H, 2, square_root=True)` for dense X (SK:85-129, beta==2 branch:
    res = squared_norm(X - W·H)/2, returned as sqrt(2·res)).  squared_norm = dot(ravel, ravel)
    (`sklearn/utils/extmath.py:19-44`)."""
    R = np.ravel(X - np.dot(W, H), order="K")
    res = np.dot(R, R) / 2.0
    return np.sqrt(2 * res)


# --------------------------------------------------------------------------------------------
# a1 / a2: the two multiplicative updates (beta_loss == 2 branches)
# --------------------------------------------------------------------------------------------
def update_w(X, W, H, l1_reg_W=0.0, l2_reg_W=0.0, HHt=None, XHt=None, update_H=True):
    """`_multiplicative_update_w`, Frobenius branch (SK:526-631).

    numerator = X·Hᵀ (SK:543; copied when update_H is False, SK:544-550), denominator = W·(H·Hᵀ)
    (SK:553-554), + l1 (SK:616-617), + l2·W (SK:618-619), zeros → EPSILON (SK:620),
    numerator /= denominator; W *= numerator (SK:622-629).  W is updated in place.
    """
    if XHt is None:
        XHt = np.dot(X, H.T)
    numerator = XHt if update_H else XHt.copy()
    if HHt is None:
        HHt = np.dot(H, H.T)
    denominator = np.dot(W, HHt)
    if l1_reg_W > 0:
        denominator += l1_reg_W
    if l2_reg_W > 0:
        denominator = denominator + l2_reg_W * W
    denominator[denominator == 0] = EPSILON
    numerator /= denominator
    W *= numerator
    return W, HHt, XHt


def update_h(X, W, H, l1_reg_H=0.0, l2_reg_H=0.0):
    """`_multiplicative_update_h`, Frobenius branch (SK:634-728).

    numerator = Wᵀ·X (SK:639), denominator = multi_dot([Wᵀ, W, H]) = (WᵀW)·H (SK:640),
    + l1 (SK:702-703), + l2·H (SK:704-705), zeros → EPSILON (SK:706), H *= numerator/denominator
    (SK:722-726).  Returns the updated H (in place).
    """
    numerator = np.dot(W.T, X)
    denominator = np.linalg.multi_dot([W.T, W, H])
    if l1_reg_H > 0:
        denominator += l1_reg_H
    if l2_reg_H > 0:
        denominator = denominator + l2_reg_H * H
    denominator[denominator == 0] = EPSILON
    delta_H = numerator
    delta_H /= denominator
    H *= delta_H
    return H


# --------------------------------------------------------------------------------------------
# a4: driver loop
# --------------------------------------------------------------------------------------------
def mu_fit(X, W, H, max_iter=200, tol=1e-4, l1_reg_W=0.0, l1_reg_H=0.0, l2_reg_W=0.0,
           l2_reg_H=0.0, update_H=True, return_errors=False):
    """`_fit_multiplicative_update` for beta_loss='frobenius' (SK:731-893; loop SK:831-884).

    W then H each iteration; every 10 iterations when tol > 0 the Frobenius error is computed and
    the loop stops when (previous − error)/error_at_init < tol (SK:872-884).  Inputs are copied.
    Returns (W, H, n_iter) or, with return_errors, (W, H, n_iter, [(n_iter, error), ...]).
    """
    W = np.array(W, copy=True)
    H = np.array(H, copy=True)
    error_at_init = frobenius_error(X, W, H)
    previous_error = error_at_init
    errors = [(0, float(error_at_init))]
    HHt = XHt = None
    n_iter = 0
    for n_iter in range(1, max_iter + 1):
        W, HHt, XHt = update_w(X, W, H, l1_reg_W, l2_reg_W, HHt=HHt, XHt=XHt,
                               update_H=update_H)
        if update_H:
            H = update_h(X, W, H, l1_reg_H, l2_reg_H)
            HHt = XHt = None
        if tol > 0 and n_iter % 10 == 0:
            error = frobenius_error(X, W, H)
            errors.append((n_iter, float(error)))
            if (previous_error - error) / error_at_init < tol:
                break
            previous_error = error
    if return_errors:
        return W, H, n_iter, errors
    return W, H, n_iter


def compute_regularization(n_samples, n_features, alpha_W=0.0, alpha_H="same", l1_ratio=0.0):
    """`_BaseNMF._compute_regularization` (SK:1254-1265)."""
    alpha_H = alpha_W if alpha_H == "same" else alpha_H
    l1_reg_W = n_features * alpha_W * l1_ratio
    l1_reg_H = n_samples * alpha_H * l1_ratio
    l2_reg_W = n_features * alpha_W * (1.0 - l1_ratio)
    l2_reg_H = n_samples * alpha_H * (1.0 - l1_ratio)
    return l1_reg_W, l1_reg_H, l2_reg_W, l2_reg_H


def transform_init(X, n_components):
    """W start for update_H=False with solver='mu': filled with sqrt(X.mean()/k) (SK:1228-1232)."""
    avg = np.sqrt(X.mean() / n_components)
    return np.full((X.shape[0], n_components), avg, dtype=X.dtype)


# --------------------------------------------------------------------------------------------
# sharding algebra (row e): A = WᵀX and B = WᵀW are sums over row blocks
# --------------------------------------------------------------------------------------------
def sharded_accumulators(X, W, n_shards):
    """Per-shard (A_p, B_p) for contiguous row shards; their sum equals (WᵀX, WᵀW)."""
    bounds = np.linspace(0, X.shape[0], n_shards + 1).astype(np.int64)
    out = []
    for p in range(n_shards):
        lo, hi = bounds[p], bounds[p + 1]
        out.append((W[lo:hi].T @ X[lo:hi], W[lo:hi].T @ W[lo:hi]))
    return out


def update_h_from_accumulators(A, B, H, l1_reg_H=0.0, l2_reg_H=0.0):
    """`update_h` (SK:634-728) expressed on the reduced accumulators A = WᵀX, B = WᵀW — the form the
    sharded path applies after the all-reduce."""
    denominator = B @ H
    if l1_reg_H > 0:
        denominator += l1_reg_H
    if l2_reg_H > 0:
        denominator = denominator + l2_reg_H * H
    denominator[denominator == 0] = EPSILON
    return H * (A / denominator)


def normalise(W, H, norm="l2"):
    """Normalisation projection (build spec, no sklearn function): unit-norm rows
    of H with the scales folded into the columns of W, so W @ H is unchanged.  All-zero rows keep
    scale 1.  Returns (W', H', s)."""
    H = np.asarray(H, dtype=np.float64)
    if norm == "l1":
        s = np.abs(H).sum(axis=1)
    elif norm == "l2":
        s = np.sqrt((H * H).sum(axis=1))
    elif norm == "max":
        s = np.abs(H).max(axis=1)
    else:
        raise ValueError(norm)
    s = np.where(s > 0, s, 1.0)
    return np.asarray(W, dtype=np.float64) * s[None, :], H / s[:, None], s
