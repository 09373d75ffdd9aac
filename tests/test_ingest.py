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
        load_spectra(tmp_path / "x.h5", device="cpu")


def _write_nc(path, cube, dims=("wavelength", "y", "x"), scale=None, offset=None, fill=None, dtype="f4"):
    from scipy.io import netcdf_file
    with netcdf_file(str(path), "w", version=2) as nc:
        for d, n in zip(dims, cube.shape):
            nc.createDimension(d, n)
        if "wavelength" in dims:
            nc.createVariable("wavelength", "f4", ("wavelength",))[:] = np.arange(cube.shape[0]) * 5 + 350.0
        v = nc.createVariable("a", dtype, dims)
        if scale is not None:
            v.scale_factor = scale
        if offset is not None:
            v.add_offset = offset
        if fill is not None:
            v._FillValue = fill
        v[:] = cube


def test_netcdf3_cube_round_trip(tmp_path):
    """An IOP cube a(wavelength, y, x) in a netCDF-3 file: samples = pixels in C order, columns =
    wavelengths; chunking over the leading sample dimension reads back exactly."""
    X = iop_spectra(6 * 7, 81, seed=4, dtype=np.float32)            # 42 pixels x 81 bands
    cube = X.reshape(6, 7, 81).transpose(2, 0, 1).copy()           # (wavelength, y, x)
    p = tmp_path / "iop.nc"
    _write_nc(p, cube)
    for chunk in (1, 7, 15, 1000):
        t = load_spectra(p, device="cpu", chunk_rows=chunk)
        np.testing.assert_array_equal(t.numpy(), X)
    # the feature dimension named explicitly, a (y, x, band) layout
    q = tmp_path / "iop2.nc"
    _write_nc(q, X.reshape(6, 7, 81), dims=("y", "x", "band"))
    np.testing.assert_array_equal(load_spectra(q, device="cpu", feature_dim="band").numpy(), X)


def test_netcdf3_scale_offset_and_fill(tmp_path):
    X = iop_spectra(20, 81, seed=5, dtype=np.float64)
    cube = X.reshape(4, 5, 81).transpose(2, 0, 1)
    packed = np.round((cube - 0.001) / 1e-4).astype(np.int16)     # packed shorts, as ocean products ship
    packed[:, 1, 2] = -32767                                       # one land pixel
    p = tmp_path / "packed.nc"
    _write_nc(p, packed, scale=1e-4, offset=0.001, fill=-32767, dtype="h")
    with pytest.raises(ValueError, match="NaN"):
        load_spectra(p, device="cpu", dtype=np.float64)
    t, rows = load_spectra(p, device="cpu", dtype=np.float64, drop_invalid=True)
    assert t.shape == (19, 81) and 1 * 5 + 2 not in rows.tolist() and len(rows) == 19
    sc, off = float(np.float32(1e-4)), float(np.float32(0.001))  # the file stores the attributes as floats
    ref = (packed.transpose(1, 2, 0).reshape(20, 81).astype(np.float64) * sc + off)[rows]
    np.testing.assert_allclose(t.numpy(), ref, rtol=0, atol=1e-15)
    assert np.abs(np.delete(packed.reshape(81, -1), 7, axis=1)).max() < 32000
    np.testing.assert_allclose(t.numpy(), X[rows], atol=6e-5)
