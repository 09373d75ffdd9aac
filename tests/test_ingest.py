"""Spectra ingest (cnmf_amd/ingest.py) on the host: .npy (memory-mapped) and
Parquet (row groups crossing the chunk boundaries) read back exactly; malformed inputs are refused."""
import numpy as np
import pytest

from cnmf_amd.ingest import load_spectra, save_parquet
from cnmf_amd.synthetic import iop_spectra


@pytest.mark.parametrize("chunk_rows", [700, 5000, 1])
def test_parquet_round_trip(tmp_path, chunk_rows):
    X = iop_spectra(2345 if chunk_rows > 1 else 17, 81, seed=2, dtype=np.float32)
    wl = np.arange(350, 755, 5)
    p = tmp_path / "iop.parquet"
    save_parquet(p, X, wavelengths=wl, row_group_rows=1000)
    t = load_spectra(p, device="cpu", chunk_rows=chunk_rows)
    np.testing.assert_array_equal(t.numpy(), X)
    # a column subset, in the caller's order
    cols = [str(w) for w in wl[[3, 1, 40]]]
    t2 = load_spectra(p, device="cpu", columns=cols, dtype=np.float64)
    np.testing.assert_array_equal(t2.numpy(), X[:, [3, 1, 40]].astype(np.float64))


def test_npy_round_trip(tmp_path):
    X = iop_spectra(1000, 81, seed=3, dtype=np.float64)
    p = tmp_path / "iop.npy"
    np.save(p, X)
    np.testing.assert_array_equal(load_spectra(p, device="cpu", dtype=np.float64, chunk_rows=333).numpy(), X)
    np.testing.assert_array_equal(load_spectra(p, device="cpu", chunk_rows=333).numpy(), X.astype(np.float32))


def test_refusals(tmp_path):
    p = tmp_path / "bad.npy"
    np.save(p, np.zeros(5))
    with pytest.raises(ValueError, match="2-D"):
        load_spectra(p, device="cpu")
    X = np.ones((10, 3), np.float32)
    X[4, 1] = np.nan
    q = tmp_path / "nan.parquet"
    save_parquet(q, X)
    with pytest.raises(ValueError, match="NaN"):
        load_spectra(q, device="cpu")
    with pytest.raises(ValueError, match="no column"):
        load_spectra(q, device="cpu", columns=["f0", "nope"])
    with pytest.raises(ValueError, match="unsupported"):
        load_spectra(tmp_path / "x.nc", device="cpu")
