"""Spectra from files into HBM: the data format on the caller's side of the
hot path.

The reference declares xarray + h5netcdf for its IOP cubes (`/root/reference/setup.py:28`); neither
(nor h5py / netCDF4) is in this image, so netCDF is not read here.  What is read:

* `.npy` (memory-mapped, `allow_pickle=False`): an (n_samples, n_features) array;
* Parquet (pyarrow): one column per wavelength / feature, one row per sample, read row group by
  row group (`columns=` selects and orders the features).

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


def load_spectra(path, *, columns=None, dtype=np.float32, device=None, chunk_rows=1 << 18):
    """Read an (n_samples, n_features) spectra file into a contiguous tensor on `device` (default:
    the current HIP device; "cpu" gives a host tensor).  `dtype`: np.float32 (default) or
    np.float64.  Raises ValueError for a malformed file or non-finite values."""
    dtype = np.dtype(dtype)
    if dtype not in (np.float32, np.float64):
        raise ValueError(f"dtype must be float32 or float64, got {dtype}")
    ext = os.path.splitext(str(path))[1].lower()
    if ext == ".npy":
        n, f, gen = _row_chunks_npy(path, columns)
    elif ext in (".parquet", ".pq"):
        n, f, gen = _row_chunks_parquet(path, columns)
    else:
        raise ValueError(f"{path}: unsupported format {ext!r} (.npy or .parquet; netCDF readers are not "
                         "in this image)")
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
