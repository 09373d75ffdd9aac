"""ctypes binding of libcnmf_hip.so (C ABI declared in include/cnmf_hip.h).

The library is loaded AFTER `import torch`, so the HIP runtime torch already mapped
(libamdhip64.so.7 in torch/lib) is the one the library binds to: one runtime, one set of streams
per process ("Two HIP runtimes").  There is no CPU fallback: if the library is
missing or fails to load, every entry point raises `HipLibraryError`.
"""
from __future__ import annotations

import ctypes
import os
import re

__all__ = ["HipLibraryError", "load", "lib_path", "header_path", "declared_symbols", "check",
           "F32", "F64", "BF16", "PASS_UPDATE_W", "PASS_ACCUMULATE", "PASS_LOSS"]

F32, F64, BF16 = 0, 1, 2
PASS_UPDATE_W, PASS_ACCUMULATE, PASS_LOSS = 1, 2, 4

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class HipLibraryError(RuntimeError):
    """The HIP extension is missing, failed to load, or a call returned an error status."""


def lib_path() -> str:
    return os.environ.get("CNMF_HIP_LIB", os.path.join(_HERE, "libcnmf_hip.so"))


def header_path() -> str:
    return os.path.join(os.path.dirname(_HERE), "include", "cnmf_hip.h")


def declared_symbols() -> list[str]:
    """Every function the public header declares (the ABI test checks the .so exports them)."""
    with open(header_path()) as f:
        text = f.read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\**\s+\**(cnmf_[a-z_0-9]+)\(", text, re.M)))


_vp, _i32, _i64, _f64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_double

_SIGS = {
    "cnmf_abi_version": (_i32, []),
    "cnmf_last_error": (ctypes.c_char_p, []),
    "cnmf_padded_k": (_i32, [_i32]),
    "cnmf_pass_blocks": (_i64, [_i64, _i32, _i32, _i32]),
    "cnmf_stage_doubles": (_i64, [_i32]),
    "cnmf_mu_sample_pass": (_i32, [_vp, _i32, _vp, _vp, _vp, _vp, _i64, _i32, _i32, _f64, _f64,
                                   _i32, _vp]),
    "cnmf_reduce_partials": (_i32, [_vp, _i64, _i32, _vp, _vp, _vp, _vp]),
    "cnmf_basis_update": (_i32, [_vp, _vp, _vp, _vp, _i32, _i32, _f64, _f64, _i32, _vp, _vp]),
    "cnmf_reduce_update": (_i32, [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _i32, _f64, _f64,
                                  _vp, _vp]),
    "cnmf_mu_iterations": (_i32, [_i32, _vp, _i32, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp,
                                  _vp, _i64, _i32, _i32, _f64, _f64, _f64, _f64, _i32, _vp, _i32, _vp]),
    "cnmf_counter_words": (_i64, []),
    "cnmf_wmu_pass_blocks": (_i64, [_i64, _i32, _i32]),
    "cnmf_wmu_sample_pass": (_i32, [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i32, _i32, _i32, _vp]),
    "cnmf_wmu_basis_update": (_i32, [_vp, _vp, _i32, _i32, _vp]),
    "cnmf_wmu_persistent": (_i32, [_i64, _i32, _i32]),
    "cnmf_wmu_iterations": (_i32, [_i32, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _i64, _i32, _i32,
                                   _vp, _i32, _vp]),
    "cnmf_wmu_iterations_multi": (_i32, [_i32, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _i64, _i32,
                                         _i32, _vp, _vp, _i32, _vp]),
    "cnmf_counter_err_word": (_i32, []),
    "cnmf_mu_persistent": (_i32, [_i64, _i32, _i32, _i32]),
    "cnmf_als_table_doubles": (_i32, []),
    "cnmf_als_prepare": (_i32, [_vp, _vp, _vp, _vp, _i32, _i32, _f64, _vp]),
    "cnmf_als_sample_pass": (_i32, [_vp, _i32, _vp, _vp, _vp, _vp, _i64, _i32, _i32, _f64, _i32, _vp]),
    "cnmf_als_basis_update": (_i32, [_vp, _vp, _vp, _vp, _vp, _i32, _i32, _f64, _f64, _vp]),
    "cnmf_als_persistent": (_i32, [_i64, _i32, _i32, _i32]),
    "cnmf_als_iterations": (_i32, [_i32, _vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _i64,
                                   _i32, _i32, _f64, _f64, _vp, _i32, _vp]),
    "cnmf_als_iterations_multi": (_i32, [_i32, _vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp,
                                         _i64, _i32, _i32, _f64, _f64, _vp, _vp, _i32, _vp]),
    "cnmf_als_persist_workgroups": (_i64, [_i64, _i32, _i32, _i32, _i32]),
    "cnmf_als_fit_tol": (_i32, [_i32, _vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp,
                                _i64, _i32, _i32, _f64, _f64, _vp, _vp, _i32, _vp]),
    "cnmf_normalise": (_i32, [_vp, _i32, _vp, _vp, _vp, _vp, _i64, _i32, _i32, _i32, _vp]),
    "cnmf_mu_shard_step": (_i32, [_vp, _i32, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _i64, _i32,
                                  _i32, _f64, _f64, _f64, _f64, _i32, _i32, _vp]),
    "cnmf_xbuf_bytes": (_i64, [_i32]),
    "cnmf_xbuf_handle_bytes": (_i32, []),
    "cnmf_device_pci_bus_id": (_i32, [_i32, ctypes.c_char_p, _i32]),
    "cnmf_device_can_access_peer": (_i32, [_i32, _i32]),
    "cnmf_enable_peer_access": (_i32, [_i32, _i32]),
    "cnmf_tolctl_doubles": (_i32, [_i32]),
    "cnmf_mu_fit_tol": (_i32, [_i32, _vp, _i32, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _i64, _i32,
                               _i32, _f64, _f64, _f64, _f64, _i32, _vp, _vp, _i32, _vp]),
    "cnmf_persist_workgroups": (_i64, [_i64, _i32, _i32, _i32, _i32, _i32]),
    "cnmf_xbuf_alloc": (_i32, [_i32, ctypes.POINTER(_vp), _vp]),
    "cnmf_xbuf_open": (_i32, [_vp, ctypes.POINTER(_vp)]),
    "cnmf_xbuf_close": (_i32, [_vp]),
    "cnmf_xbuf_free": (_i32, [_vp]),
    "cnmf_xctl_words": (_i64, [_i32]),
    "cnmf_xctl_init": (_i32, [_vp, _vp, _i32, _i32]),
    "cnmf_init_gram_rows": (_i64, [_i64]),
    "cnmf_init_gram": (_i32, [_vp, _i32, _i64, _i32, _vp, _i64, _vp]),
    "cnmf_init_xm": (_i32, [_vp, _i32, _i64, _i32, _i32, _vp, _vp, _vp]),
    "cnmf_init_stats_rows": (_i64, [_i64]),
    "cnmf_init_stats": (_i32, [_vp, _i64, _i32, _vp, _i64, _vp]),
    "cnmf_init_fill": (_i32, [_vp, _i64, _i32, _vp, _vp, _vp, _f64, _f64, _vp, _i32, _vp]),
    "cnmf_persist_describe": (_i32, [_i64, _i32, _i32, _i32, _i32, ctypes.c_char_p, _i32]),
    "cnmf_host_register": (_i32, [_vp, _i64]),
    "cnmf_host_unregister": (_i32, [_vp]),
    "cnmf_copy_h2d_async": (_i32, [_vp, _vp, _i64, _vp]),
    "cnmf_mu_iterations_multi": (_i32, [_i32, _vp, _i32, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp,
                                        _i64, _i32, _i32, _f64, _f64, _f64, _f64, _vp, _i32, _vp, _i32,
                                        _vp]),
}


def load():
    """Load (once) and return the ctypes handle; raises HipLibraryError when unavailable."""
    global _LIB
    if _LIB is not None:
        return _LIB
    import torch  # noqa: F401  — map torch's HIP runtime first (see module docstring)

    path = lib_path()
    if not os.path.exists(path):
        raise HipLibraryError(
            f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `python -m cnmf_amd.build` (hipcc --offload-arch=gfx950). There is no CPU fallback.")
    try:
        lib = ctypes.CDLL(path)
    except OSError as e:
        raise HipLibraryError(f"failed to load {path}: {e}") from e
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = lib
    return lib


def check(status: int, what: str = "") -> int:
    """Raise HipLibraryError for a negative status, with the library's thread-local message."""
    if status < 0:
        msg = load().cnmf_last_error().decode(errors="replace")
        raise HipLibraryError(f"{what or 'cnmf call'} failed ({status}): {msg}")
    return status
