"""The host initialisation (cnmf_amd/init.py, SK:221-373 over extmath.py:287-604) against
sklearn's own `_initialize_nmf` outputs (tests/golden/init_*.npz, make_golden.py:init_cases):
NNDSVD / NNDSVDA / NNDSVDAR in fp64 and fp32, a k = 8 case and init=None's default.  The host
restatement keeps sklearn's arithmetic op for op, so the bar is equality up to BLAS summation
order (1e-12 fp64, 1e-6 fp32 relative Frobenius; in practice bit-identical here)."""
import numpy as np
import pytest

from golden_io import init_names, load_init, rel_fro


@pytest.mark.parametrize("name", init_names())
def test_host_init_matches_sklearn(name):
    from cnmf_amd.init import initialize_nmf
    case = load_init(name)
    kw = case["kwargs"]
    X = case["X"]
    W, H = initialize_nmf(X, kw["n_components"], init=kw["init"], random_state=kw["random_state"])
    assert W.dtype == case["W"].dtype and H.dtype == case["H"].dtype
    tol = 1e-12 if X.dtype == np.float64 else 1e-6
    assert rel_fro(W, case["W"]) <= tol and rel_fro(H, case["H"]) <= tol, (rel_fro(W, case["W"]),
                                                                        rel_fro(H, case["H"]))
    # the zero pattern decides NNDSVDAR's random fill order: it must be the same
    np.testing.assert_array_equal(W == 0, case["W"] == 0)


def test_init_goldens_cover_the_family():
    inits = {load_init(n)["kwargs"]["init"] for n in init_names()}
    dts = {str(load_init(n)["X"].dtype) for n in init_names()}
    assert {"nndsvd", "nndsvda", "nndsvdar", None} <= inits and dts == {"float32", "float64"}


@pytest.mark.parametrize("name", ["tall_default_float32", "tall_default_tol_float32"])
def test_tall_default_start_is_sklearns(name):
    """The start cnmf's default fit takes for a tall float32 X (init_device='auto': the host
    restatement) is sklearn's _initialize_nmf output bit for bit (X regenerated from its seed)."""
    import hashlib
    import json
    import os
    from cnmf_amd.init import initialize_nmf
    from cnmf_amd.synthetic import iop_spectra
    from golden_io import GOLDEN
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)
    X = iop_spectra(int(z["n_rows"]), 81, seed=int(z["seed"]), dtype=np.float32)
    assert hashlib.sha256(X.tobytes()).hexdigest() == str(z["x_sha256"])
    kw = json.loads(str(z["kwargs"]))
    W, H = initialize_nmf(X, kw["n_components"], init=None, random_state=kw["random_state"])
    np.testing.assert_array_equal(W, z["W_init"])
    np.testing.assert_array_equal(H, z["H_init"])
