"""Host-side initialisation of (W, H): the non-hot part of row (a5), run once per fit.

Restates sklearn 1.7.2's `_initialize_nmf` (SK:221-373) — 'random' (SK:303-314) and the
NNDSVD family (SK:317-373) — together with the randomized SVD it calls
(`sklearn/utils/extmath.py`: `_randomized_range_finder` :287-357, `_randomized_svd` :530-604,
`svd_flip` :900-953) op for op in NumPy/SciPy, so a NumPy X gives the same (W0, H0) as sklearn
for the same random_state.  The hot loop never runs here; the GPU NNDSVD is
`cnmf_amd.gpu_init`.

Attribution: the NNDSVD and randomized-SVD code below is a transcription of scikit-learn's
(BSD 3-Clause License, Copyright (c) 2007-2024 The scikit-learn developers; the license text ships
with scikit-learn as sklearn/COPYING): keeping its arithmetic op for op is what makes the host init
bit-identical to the reference's declared solver library.
"""
from __future__ import annotations

from functools import partial
from math import sqrt

import numpy as np
from scipy import linalg

from .synthetic import random_init

__all__ = ["initialize_nmf", "randomized_svd"]


def _check_random_state(seed):
    if seed is None or seed is np.random:
        return np.random.mtrand._rand
    if isinstance(seed, (int, np.integer)):
        return np.random.RandomState(seed)
    if isinstance(seed, np.random.RandomState):
        return seed
    raise ValueError(f"{seed!r} cannot be used to seed a numpy.random.RandomState instance")


def _svd_flip(u, v, u_based_decision=True):
    """extmath.py:900-953."""
    if u_based_decision:
        max_abs_u_cols = np.argmax(np.abs(u.T), axis=1)
        shift = np.arange(u.T.shape[0])
        indices = max_abs_u_cols + shift * u.T.shape[1]
        signs = np.sign(np.take(np.reshape(u.T, (-1,)), indices, axis=0))
        u *= signs[np.newaxis, :]
        v *= signs[:, np.newaxis]
    else:
        max_abs_v_rows = np.argmax(np.abs(v), axis=1)
        shift = np.arange(v.shape[0])
        indices = max_abs_v_rows + shift * v.shape[1]
        signs = np.sign(np.take(np.reshape(v, (-1,)), indices, axis=0))
        u *= signs[np.newaxis, :]
        v *= signs[:, np.newaxis]
    return u, v


def _range_finder(A, size, n_iter, random_state):
    """extmath.py:287-357 (NumPy branch: LU normaliser when n_iter > 2, else none)."""
    Q = random_state.normal(size=(A.shape[1], size))
    if np.issubdtype(A.dtype, np.floating):
        Q = Q.astype(A.dtype, copy=False)
    if n_iter <= 2:
        normalizer = lambda x: (x, None)  # noqa: E731
    else:
        normalizer = partial(linalg.lu, permute_l=True, check_finite=False)
    qr_normalizer = partial(linalg.qr, mode="economic", check_finite=False)
    for _ in range(n_iter):
        Q, _ = normalizer(A @ Q)
        Q, _ = normalizer(A.T @ Q)
    Q, _ = qr_normalizer(A @ Q)
    return Q


def randomized_svd(M, n_components, n_oversamples=10, n_iter="auto", random_state=None):
    """extmath.py:530-604 with transpose='auto', flip_sign=True, lapack driver gesdd."""
    random_state = _check_random_state(random_state)
    n_random = n_components + n_oversamples
    n_samples, n_features = M.shape
    if n_iter == "auto":
        n_iter = 7 if n_components < 0.1 * min(M.shape) else 4
    transpose = n_samples < n_features
    if transpose:
        M = M.T
    Q = _range_finder(M, n_random, n_iter, random_state)
    B = Q.T @ M
    Uhat, s, Vt = linalg.svd(B, full_matrices=False, lapack_driver="gesdd")
    del B
    U = Q @ Uhat
    if not transpose:
        U, Vt = _svd_flip(U, Vt)
    else:
        U, Vt = _svd_flip(U, Vt, u_based_decision=False)
    if transpose:
        return Vt[:n_components, :].T, s[:n_components], U[:, :n_components].T
    return U[:, :n_components], s[:n_components], Vt[:n_components, :]


def _norm(x):
    x = np.ravel(x, order="K")
    return sqrt(np.dot(x, x))


def initialize_nmf(X, n_components, init=None, eps=1e-6, random_state=None):
    """SK:221-373."""
    if X.min() < 0:
        raise ValueError("Negative values in data passed to NMF initialization.")
    n_samples, n_features = X.shape
    if init is not None and init != "random" and n_components > min(n_samples, n_features):
        raise ValueError("init = '{}' can only be used when "
                         "n_components <= min(n_samples, n_features)".format(init))
    if init is None:
        init = "nndsvda" if n_components <= min(n_samples, n_features) else "random"
    if init == "random":
        return random_init(X, n_components, _check_random_state(random_state))

    U, S, V = randomized_svd(X, n_components, random_state=random_state)
    W = np.zeros_like(U)
    H = np.zeros_like(V)
    W[:, 0] = np.sqrt(S[0]) * np.abs(U[:, 0])
    H[0, :] = np.sqrt(S[0]) * np.abs(V[0, :])
    for j in range(1, n_components):
        x, y = U[:, j], V[j, :]
        x_p, y_p = np.maximum(x, 0), np.maximum(y, 0)
        x_n, y_n = np.abs(np.minimum(x, 0)), np.abs(np.minimum(y, 0))
        x_p_nrm, y_p_nrm = _norm(x_p), _norm(y_p)
        x_n_nrm, y_n_nrm = _norm(x_n), _norm(y_n)
        m_p, m_n = x_p_nrm * y_p_nrm, x_n_nrm * y_n_nrm
        if m_p > m_n:
            u, v, sigma = x_p / x_p_nrm, y_p / y_p_nrm, m_p
        else:
            u, v, sigma = x_n / x_n_nrm, y_n / y_n_nrm, m_n
        lbd = np.sqrt(S[j] * sigma)
        W[:, j] = lbd * u
        H[j, :] = lbd * v
    W[W < eps] = 0
    H[H < eps] = 0
    if init == "nndsvd":
        pass
    elif init == "nndsvda":
        avg = X.mean()
        W[W == 0] = avg
        H[H == 0] = avg
    elif init == "nndsvdar":
        rng = _check_random_state(random_state)
        avg = X.mean()
        W[W == 0] = abs(avg * rng.standard_normal(size=len(W[W == 0])) / 100)
        H[H == 0] = abs(avg * rng.standard_normal(size=len(H[H == 0])) / 100)
    else:
        raise ValueError("Invalid init parameter: got %r instead of one of %r"
                         % (init, (None, "random", "nndsvd", "nndsvda", "nndsvdar")))
    return W, H
