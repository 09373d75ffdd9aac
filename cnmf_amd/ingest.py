"""Spectra from files into HBM: the data format on the caller's side of the
hot path.

The reference declares xarray + h5netcdf for its IOP cubes (`/root/reference/setup.py:25,27`);
neither (nor h5py / netCDF4) is in this image, so netCDF-4 / HDF5 files are not read here.  What is
read:

* `.npy` (memory-mapped, `allow_pickle=False`): an (n_samples, n_features) array;
* Parquet (pyarrow): one column per wavelength / feature, one row per sample, read row group by
  row group (`columns=` selects and orders the features);
* netCDF-3 classic / 64-bit offset (`.nc`, scipy.io.netcdf_file, memory-mapped): one variable of an
  IOP cube, e.g. a(wavelength, y, x); the feature (wavelength) dimension becomes the columns and
  every other dimension is flattened into samples in C order (`variable=`, `feature_dim=`;
  scale_factor / add_offset applied; _FillValue / missing_value pixels are refused, or dropped with
  `drop_invalid=True`, which also returns the kept rows' flat sample indices).

Either way the rows stream through two pinned host buffers of `chunk_rows` rows into one
preallocated device tensor: chunk i+1 is converted into one pinned buffer while chunk i's
host-to-device copy (non_blocking, on a side stream) drains from the other; a buffer is reused only
after its copy's event has completed.  Host memory in use stays at 2 chunks whatever the file
size, and the copies overlap the file reads.  The result is what `cnmf_amd.factorise` and the
plans take (row-major fp32 / fp64, contiguous).
"""
from __future__ import annotations

import os

import numpy as np
import torch

__all__ = ["load_spectra", "save_parquet"]


def _row_chunks_npy(path, columns):
    arr = np.load(path, mmap_mode="r", allow_pickle=False)
    if arr.ndim != 2:
        raise ValueError(f"{path}: expected a 2-D array (samples x features), got shape {arr.shape}")
    if columns is not None:
        raise ValueError("columns= applies to Parquet files")
    n, f = arr.shape

    def gen(chunk_rows):
        for lo in range(0, n, chunk_rows):
            yield arr[lo:lo + chunk_rows]
    return n, f, gen


def _row_chunks_parquet(path, columns):
    import pyarrow.parquet as pq
    pf = pq.ParquetFile(path)
    names = list(columns) if columns is not None else list(pf.schema_arrow.names)
    missing = [c for c in names if c not in pf.schema_arrow.names]
    if missing:
        raise ValueError(f"{path}: no column(s) {missing}")
    n, f = pf.metadata.num_rows, len(names)

    def gen(chunk_rows):
        for batch in pf.iter_batches(batch_size=chunk_rows, columns=names):
            yield np.stack([batch.column(i).to_numpy(zero_copy_only=False) for i in range(f)], axis=1)
    return n, f, gen


_FEATURE_DIM_NAMES = ("wavelength", "wavelengths", "lambda", "wl", "wave", "band", "bands", "feature")


def _netcdf_variable(path, variable, feature_dim):
    from scipy.io import netcdf_file
    nc = netcdf_file(str(path), "r", mmap=True, maskandscale=False)
    cands = {k: v for k, v in nc.variables.items() if len(v.dimensions) >= 2}
    if variable is None:
        if len(cands) != 1:
            raise ValueError(f"{path}: name the variable (variable=...) among {sorted(cands) or 'none'}")
        variable = next(iter(cands))
    if variable not in nc.variables:
        raise ValueError(f"{path}: no variable {variable!r}")
    var = nc.variables[variable]
    dims = list(var.dimensions)
    if len(dims) < 1:
        raise ValueError(f"{path}: variable {variable!r} is a scalar")
    if feature_dim is None:
        named = [d for d in dims if d.lower() in _FEATURE_DIM_NAMES]
        feature_dim = named[0] if len(named) == 1 else dims[-1]
    if feature_dim not in dims:
        raise ValueError(f"{path}: {variable!r} has no dimension {feature_dim!r} (dims {dims})")
    return nc, var, dims.index(feature_dim)


def _row_chunks_netcdf(path, columns, variable, feature_dim):
    if columns is not None:
        raise ValueError("columns= applies to Parquet files")
    nc, var, fd = _netcdf_variable(path, variable, feature_dim)
    data = np.moveaxis(var.data, fd, -1)  # a view of the memory map: samples..., features
    f = data.shape[-1]
    per_lead = int(np.prod(data.shape[1:-1])) if data.ndim > 2 else 1
    n = int(np.prod(data.shape[:-1])) if data.ndim > 1 else 1
    att = var._attributes
    scale = float(att.get("scale_factor", 1.0))
    offset = float(att.get("add_offset", 0.0))
    fills = [att[k] for k in ("_FillValue", "missing_value") if k in att]

    def gen(chunk_rows):
        lead = max(1, chunk_rows // max(per_lead, 1))
        for lo in range(0, data.shape[0], lead):
            raw = np.asarray(data[lo:lo + lead]).reshape(-1, f)
            part = raw.astype(np.float64)
            bad = np.zeros(raw.shape, dtype=bool)
            for fv in fills:
                bad |= raw == np.asarray(fv, dtype=raw.dtype)
            if scale != 1.0:
                part *= scale
            if offset != 0.0:
                part += offset
            part[bad] = np.nan
            yield part
    return n, f, gen, nc


def load_spectra(path, *, columns=None, dtype=np.float32, device=None, chunk_rows=1 << 18,
                 variable=None, feature_dim=None, drop_invalid=False):
    """Read an (n_samples, n_features) spectra file into a contiguous tensor on `device` (default:
    the current HIP device; "cpu" gives a host tensor).  `dtype`: np.float32 (default) or
    np.float64.  netCDF-3 (.nc): `variable` (default: the only variable with >= 2 dimensions),
    `feature_dim` (default: the dimension named like a wavelength, else the last one).  Raises
    ValueError for a malformed file or non-finite values; with drop_invalid=True (netCDF) the
    samples holding a fill value or a non-finite value are dropped and (tensor, kept flat sample
    indices) is returned."""
    dtype = np.dtype(dtype)
    if dtype not in (np.float32, np.float64):
        raise ValueError(f"dtype must be float32 or float64, got {dtype}")
    ext = os.path.splitext(str(path))[1].lower()
    if ext == ".nc":
        n, f, gen, nc = _row_chunks_netcdf(path, columns, variable, feature_dim)
        try:
            if drop_invalid:
                return _load_dropping_invalid(gen, f, dtype, device, chunk_rows)
            return _load(gen, n, f, dtype, device, chunk_rows, path)
        finally:
            nc.close()
    if drop_invalid:
        raise ValueError("drop_invalid= applies to netCDF files")
    if ext == ".npy":
        n, f, gen = _row_chunks_npy(path, columns)
    elif ext in (".parquet", ".pq"):
        n, f, gen = _row_chunks_parquet(path, columns)
    else:
        raise ValueError(f"{path}: unsupported format {ext!r} (.npy, .parquet or netCDF-3 .nc; "
                         "netCDF-4 / HDF5 readers are not in this image)")
    return _load(gen, n, f, dtype, device, chunk_rows, path)


def _load_dropping_invalid(gen, f, dtype, device, chunk_rows):
    """The rows of every chunk that are finite everywhere, and their flat sample indices."""
    keep, idx, lo = [], [], 0
    for part in gen(max(1, int(chunk_rows))):
        ok = np.isfinite(part).all(axis=1)
        keep.append(part[ok].astype(dtype))
        idx.append(np.nonzero(ok)[0] + lo)
        lo += part.shape[0]
    X = np.concatenate(keep) if keep else np.zeros((0, f), dtype)
    rows = np.concatenate(idx) if idx else np.zeros(0, np.int64)
    t = torch.from_numpy(np.ascontiguousarray(X))
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    return t.to(torch.device(device)), rows


def _load(gen, n, f, dtype, device, chunk_rows, path):
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    device = torch.device(device)
    tdt = torch.float32 if dtype == np.float32 else torch.float64
    out = torch.empty((n, f), dtype=tdt, device=device)
    chunk_rows = max(1, int(chunk_rows))
    if device.type == "cpu":
        lo = 0
        for part in gen(chunk_rows):
            m = part.shape[0]
            out[lo:lo + m] = torch.from_numpy(np.ascontiguousarray(part, dtype=dtype))
            lo += m
        _check_finite(out)
        return out
    side = torch.cuda.Stream(device)
    bufs = [torch.empty((chunk_rows, f), dtype=tdt, pin_memory=True) for _ in range(2)]
    done = [None, None]
    lo = 0
    with torch.cuda.device(device):
        # `out` was allocated on the current stream: the side stream's copies into it must follow
        # whatever work the caching allocator's recycled block may still have queued there
        side.wait_stream(torch.cuda.current_stream(device))
        for i, part in enumerate(gen(chunk_rows)):
            m = part.shape[0]
            b = i & 1
            if done[b] is not None:
                done[b].synchronize()  # that buffer's previous copy has drained
            bufs[b][:m].numpy()[...] = part  # convert (dtype) straight into pinned memory
            with torch.cuda.stream(side):
                out[lo:lo + m].copy_(bufs[b][:m], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(side)
            done[b] = ev
            lo += m
        torch.cuda.current_stream(device).wait_stream(side)
        side.synchronize()
    if lo != n:
        raise ValueError(f"{path}: read {lo} rows, the file declares {n}")
    _check_finite(out)
    return out


def _check_finite(t):
    if not bool(torch.isfinite(t).all()):
        raise ValueError("Input X contains NaN or infinity.")


def save_parquet(path, X, wavelengths=None, row_group_rows=1 << 16):
    """Write an (n_samples, n_features) array as Parquet, one column per feature (named by
    `wavelengths`, default "f0", "f1", ...), in row groups of `row_group_rows` rows."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    X = np.asarray(X)
    names = [str(w) for w in wavelengths] if wavelengths is not None else [f"f{i}" for i in range(X.shape[1])]
    table = pa.table({nm: X[:, i] for i, nm in enumerate(names)})
    pq.write_table(table, path, row_group_size=row_group_rows)
