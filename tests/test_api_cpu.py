"""API validation mirrors sklearn's messages (SK:68-82, SK:1194-1252) and rejects what the MI355X
path does not implement — all before any device work, so these run on CPU."""
import warnings

import numpy as np
import pytest

import cnmf
import cnmf_amd
from cnmf_amd.synthetic import iop_spectra, random_init


@pytest.fixture
def X():
    return iop_spectra(50, 81, seed=0, dtype=np.float32)


def test_drop_in_name_reexports():
    assert cnmf.factorise is cnmf_amd.factorise and cnmf.NMF is cnmf_amd.NMF
    assert cnmf.fit is cnmf_amd.factorise and cnmf.non_negative_factorization is cnmf_amd.factorise


@pytest.mark.parametrize("kw, msg", [
    (dict(solver="cd"), "multiplicative-update"),
    (dict(beta_loss="kullback-leibler"), "frobenius"),
    (dict(tol=-1.0), "'tol' parameter"),
    (dict(max_iter=0), "'max_iter' parameter"),
    (dict(alpha_W=-1.0), "'alpha_W' parameter"),
    (dict(l1_ratio=2.0), "'l1_ratio' parameter"),
    (dict(init="bogus"), "'init' parameter"),
    (dict(n_components=0), "'n_components' parameter"),
    (dict(normalise="l3"), "'normalise' parameter"),
    (dict(solver="als", alpha_W=0.1), "no alpha_W"),
    (dict(solver="als", sum_to_one=-1.0), "'sum_to_one' parameter"),
    (dict(solver="als", smoothness="x"), "'smoothness' parameter"),
    (dict(smoothness=1.0), "solver='als' only"),
])
def test_invalid_params(X, kw, msg):
    with pytest.raises(ValueError, match=msg):
        cnmf_amd.factorise(X, n_components=kw.pop("n_components", 4), **kw)


def test_custom_init_checks(X):
    W0, H0 = random_init(X, 4, 0)
    with pytest.raises(ValueError, match="wrong first dimension passed to NMF \\(input H\\)"):
        cnmf_amd.factorise(X, W0, H0[:3], n_components=4, init="custom")
    with pytest.raises(ValueError, match="wrong second dimension passed to NMF \\(input W\\)"):
        cnmf_amd.factorise(X, W0[:, :3], H0, n_components=4, init="custom")
    with pytest.raises(ValueError, match="Negative values in data passed to NMF \\(input H\\)"):
        cnmf_amd.factorise(X, W0, -H0, n_components=4, init="custom")
    with pytest.raises(ValueError, match="full of zeros"):
        cnmf_amd.factorise(X, np.zeros_like(W0), H0, n_components=4, init="custom")
    with pytest.raises(TypeError, match="same dtype as X"):
        cnmf_amd.factorise(X, W0.astype(np.float64), H0, n_components=4, init="custom")


def test_negative_X_rejected_by_init(X):
    with pytest.raises(ValueError, match="Negative values in data passed to NMF initialization"):
        cnmf_amd.factorise(-X, n_components=4, init="random")


def test_k_above_16_rejected(X):
    with pytest.raises(ValueError, match="n_components=20 is not supported"):
        cnmf_amd.factorise(X, n_components=20, init="random", random_state=0)


def test_nan_rejected(X):
    X = X.copy()
    X[0, 0] = np.nan
    with pytest.raises(ValueError, match="NaN"):
        cnmf_amd.factorise(X, n_components=4)


def test_transform_requires_fit(X):
    with pytest.raises(ValueError, match="not fitted"):
        cnmf_amd.NMF(n_components=4).transform(X)
