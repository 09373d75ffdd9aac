"""Spectra ingest into HBM (pinned double-buffered host-to-device stream)
feeding the MU path: the device tensor equals the file, and a fit on it equals a fit on the array."""
import numpy as np
import pytest

from golden_io import rel_fro

pytestmark = pytest.mark.gpu


def test_parquet_to_hbm_and_fit(tmp_path):
    import torch
    import cnmf_amd
    from cnmf_amd.ingest import load_spectra, save_parquet
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(64 * 700 + 5, 81, seed=6, dtype=np.float32)
    p = tmp_path / "iop.parquet"
    save_parquet(p, X, row_group_rows=4096)
    Xd = load_spectra(p, chunk_rows=3000)
    assert Xd.is_cuda and Xd.is_contiguous()
    assert torch.equal(Xd.cpu(), torch.from_numpy(X))
    W0, H0 = random_init(X, 4, 1)
    Wa, Ha, na = cnmf_amd.factorise(Xd, torch.from_numpy(W0).cuda(), torch.from_numpy(H0).cuda(),
                                    n_components=4, init="custom", tol=0, max_iter=50)
    Wb, Hb, nb = cnmf_amd.factorise(X, W0, H0, n_components=4, init="custom", tol=0, max_iter=50)
    assert na == nb
    assert rel_fro(Wa.cpu().numpy(), Wb) < 1e-6 and rel_fro(Ha.cpu().numpy(), Hb) < 1e-6


def test_npy_to_hbm(tmp_path):
    import torch
    from cnmf_amd.ingest import load_spectra
    from cnmf_amd.synthetic import iop_spectra
    X = iop_spectra(10_007, 300, seed=7, dtype=np.float32)
    p = tmp_path / "cube.npy"
    np.save(p, X)
    Xd = load_spectra(p, chunk_rows=1024)
    assert torch.equal(Xd.cpu(), torch.from_numpy(X))
