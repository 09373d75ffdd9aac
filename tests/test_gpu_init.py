"""GPU NNDSVD (cnmf_amd/gpu_init.py: cnmf_init_gram / _xm / _stats / _fill)
against sklearn's `_initialize_nmf` goldens (tests/golden/init_*.npz).

Tolerance: the GPU path is the same randomized SVD (same Gaussian draw, same power-iteration
count) computed in Gram form, so it differs from sklearn only by rounding: fp64 X to 1e-8 relative
Frobenius, fp32 X (sklearn runs the whole SVD in fp32) to 2e-5.  The golden cases are well
conditioned (σ_k / σ_1 >= 1e-3), where the Gram form loses nothing measurable.  NNDSVDAR's random
fill follows W's zero pattern in C order, so the zero pattern must match exactly."""
import numpy as np
import pytest

from golden_io import init_names, load_init, rel_fro

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", [n for n in init_names() if load_init(n)["kwargs"]["init"] != "random"])
def test_gpu_init_matches_sklearn(name):
    import torch
    from cnmf_amd.gpu_init import initialize_nmf_gpu
    case = load_init(name)
    kw = case["kwargs"]
    X = case["X"]
    init = kw["init"] or "nndsvda"
    W, H = initialize_nmf_gpu(torch.from_numpy(X).cuda(), kw["n_components"], init=init,
                              random_state=kw["random_state"])
    W = W.cpu().numpy()
    assert W.dtype == case["W"].dtype and H.dtype == case["H"].dtype
    tol = 1e-8 if X.dtype == np.float64 else 2e-5
    ew, eh = rel_fro(W, case["W"]), rel_fro(H, case["H"])
    print(f"{name}: rel W {ew:.2e} rel H {eh:.2e}")
    np.testing.assert_array_equal(W == 0, case["W"] == 0)
    assert ew <= tol and eh <= tol, (ew, eh)


def test_gpu_init_large_matches_host():
    """cfg2's shape (1e6 x 81 fp32, k = 4): the GPU init against the host restatement (itself
    pinned to sklearn above) run in fp64 on the same values.  sklearn's own fp32 path is NOT the
    yardstick at this size: its fp32 randomized SVD is 1.4e-3 (relative Frobenius, W; 2.5e-3 on the
    4th component) from the fp64 answer, while the GPU's fp64 Gram form is within 1e-8 of it
    (measured on CPU with the same algorithm in NumPy)."""
    import torch
    from cnmf_amd.gpu_init import initialize_nmf_gpu
    from cnmf_amd.init import initialize_nmf
    from cnmf_amd.synthetic import iop_spectra
    X = iop_spectra(1_000_000, 81, seed=4, dtype=np.float32)
    Wg, Hg = initialize_nmf_gpu(torch.from_numpy(X).cuda(), 4, init="nndsvda", random_state=0)
    Wh, Hh = initialize_nmf(X.astype(np.float64), 4, init="nndsvda", random_state=0)
    ew, eh = rel_fro(Wg.cpu().numpy(), Wh), rel_fro(Hg, Hh)
    W32, _ = initialize_nmf(X, 4, init="nndsvda", random_state=0)
    print(f"1e6 x 81: GPU vs fp64 host rel W {ew:.2e} rel H {eh:.2e}; sklearn-fp32 vs fp64 host "
          f"rel W {rel_fro(W32, Wh):.2e}")
    assert ew <= 1e-5 and eh <= 1e-5, (ew, eh)


def test_api_routes_tall_x_by_init_device():
    """init=None on X with >= GPU_INIT_MIN_ROWS rows: init_device='auto' keeps float32 X on the host
    restatement (sklearn's start, bit for bit on the same BLAS) and sends float64 X to the GPU init;
    init_device='gpu' sends float32 X to the GPU init too (its distance to sklearn's fp32 start is
    reported by tests/test_gpu_tall_default.py); the fit that follows runs either way."""
    import torch
    from cnmf_amd import api
    from cnmf_amd.init import initialize_nmf
    from cnmf_amd.synthetic import iop_spectra
    X = iop_spectra(api.GPU_INIT_MIN_ROWS + 1000, 81, seed=6, dtype=np.float32)
    W, H = api._initial_factors(X, 4, None, 3, None, False, None)
    assert isinstance(W, np.ndarray)  # auto + float32: the host restatement
    Wh32, Hh32 = initialize_nmf(X, 4, init=None, random_state=3)
    assert np.array_equal(W, Wh32) and np.array_equal(H, Hh32)
    Wg, Hg = api._initial_factors(X, 4, None, 3, None, False, None, init_device="gpu")
    assert isinstance(Wg, torch.Tensor) and Wg.is_cuda
    Wh, Hh = initialize_nmf(X.astype(np.float64), 4, init=None, random_state=3)  # see above: fp64
    assert rel_fro(Wg.cpu().numpy(), Wh) <= 1e-5 and rel_fro(Hg, Hh) <= 1e-5
    X64 = X.astype(np.float64)
    W64, _ = api._initial_factors(X64, 4, None, 3, None, False, None)
    assert isinstance(W64, torch.Tensor) and W64.is_cuda  # auto + float64: the GPU init
    assert rel_fro(W64.cpu().numpy(), Wh) <= 1e-8
    import cnmf_amd
    W1, H1, n = cnmf_amd.factorise(X, n_components=4, random_state=3, max_iter=20, tol=0.0)
    assert n == 20 and W1.shape == (X.shape[0], 4) and np.all(W1 >= 0)
    with pytest.raises(ValueError):
        cnmf_amd.factorise(X, n_components=4, init_device="tpu")
