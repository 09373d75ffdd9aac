"""Synthetic IOP absorption spectra and the sklearn random-init recipe.

The reference ships no data and no generator (`/root/reference/README.md:1-2`), so the
benchmark and parity inputs are produced here from a seeded closed-form model of absorption
by CDOM, detritus and phytoplankton:

    a(λ) = A_g·exp(−S_g(λ−440)) + A_d·exp(−S_d(λ−440)) + A_ph·[G(440,25) + 0.5·G(675,12)]

with G(μ,σ) = exp(−(λ−μ)²/(2σ²)), S_g~U(.01,.02), S_d~U(.008,.012), A_g~LogN(−3,1),
A_d~LogN(−4,1), A_ph~LogN(−3,1).  Rows are samples (samples-major, sklearn's X[N,F]).

`random_init` restates sklearn's 'random' initialisation (`sklearn/decomposition/_nmf.py:303-314`)
op for op so that a numpy X gives bit-identical (W0, H0) to sklearn: H is drawn before W from a
legacy `RandomState`, both scaled by sqrt(X.mean()/k) in X's dtype, then abs'd in place.
"""
from __future__ import annotations

import numpy as np

__all__ = ["wavelengths", "iop_spectra", "random_init"]


def wavelengths(n_features: int = 81) -> np.ndarray:
    """Wavelength grid in nm: 350..750 step 5 for F=81, 400..699 step 1 for F=300, else linspace."""
    if n_features == 81:
        return np.arange(350.0, 751.0, 5.0)
    if n_features == 300:
        return np.arange(400.0, 700.0, 1.0)
    return np.linspace(350.0, 750.0, n_features)


def _gauss(lam, mu, sigma):
    return np.exp(-((lam - mu) ** 2) / (2.0 * sigma * sigma))


def iop_spectra(n_samples: int, n_features: int = 81, seed: int = 0, dtype=np.float32,
                chunk: int = 1 << 17) -> np.ndarray:
    """Return an (n_samples, n_features) array of strictly positive synthetic absorption spectra.

    Deterministic in (n_samples, n_features, seed): parameters are drawn with
    `np.random.default_rng(seed)` in the fixed order S_g, S_d, A_g, A_d, A_ph, evaluated in fp64
    and cast to `dtype` once (so fp32/bf16 runs of the CPU oracle and the GPU see identical bits).
    """
    rng = np.random.default_rng(seed)
    s_g = rng.uniform(0.010, 0.020, n_samples)
    s_d = rng.uniform(0.008, 0.012, n_samples)
    a_g = rng.lognormal(-3.0, 1.0, n_samples)
    a_d = rng.lognormal(-4.0, 1.0, n_samples)
    a_ph = rng.lognormal(-3.0, 1.0, n_samples)
    lam = wavelengths(n_features)[None, :]
    phyto = (_gauss(lam, 440.0, 25.0) + 0.5 * _gauss(lam, 675.0, 12.0))
    out = np.empty((n_samples, n_features), dtype=dtype)
    for lo in range(0, n_samples, chunk):
        hi = min(n_samples, lo + chunk)
        blk = (a_g[lo:hi, None] * np.exp(-s_g[lo:hi, None] * (lam - 440.0))
               + a_d[lo:hi, None] * np.exp(-s_d[lo:hi, None] * (lam - 440.0))
               + a_ph[lo:hi, None] * phyto)
        out[lo:hi] = blk.astype(dtype)
    return out


def random_init(X: np.ndarray, n_components: int, random_state=None):
    """sklearn's init='random' (`_nmf.py:303-314`), restated op for op (H drawn before W)."""
    n_samples, n_features = X.shape
    avg = np.sqrt(X.mean() / n_components)
    rng = random_state if isinstance(random_state, np.random.RandomState) \
        else np.random.RandomState(random_state) if random_state is not None \
        else np.random.mtrand._rand
    H = avg * rng.standard_normal(size=(n_components, n_features)).astype(X.dtype, copy=False)
    W = avg * rng.standard_normal(size=(n_samples, n_components)).astype(X.dtype, copy=False)
    np.abs(H, out=H)
    np.abs(W, out=W)
    return W, H
