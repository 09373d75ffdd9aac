"""roctx ranges around the hot path's host-side steps (SURVEY.md §5 "Tracing / profiling").

Off unless enabled (`cnmf_amd.tracing(True)` or CNMF_ROCTX=1 in the environment): then every
stretch of iterations (one library call: one persistent launch, or a shard-step loop), every loss
evaluation and the GPU init's passes push a named range, so `rocprofv3 --marker-trace
--kernel-trace` lines the kernels up under the iterations they belong to.  The marker library is
rocprofiler-sdk's roctx (the one rocprofv3 intercepts), else roctracer's libroctx64; if neither
loads, ranges are no-ops.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

__all__ = ["tracing", "trace_range"]

_state = {"enabled": os.environ.get("CNMF_ROCTX", "0") == "1", "lib": None, "tried": False}


def _load():
    if _state["tried"]:
        return _state["lib"]
    _state["tried"] = True
    cands = ["librocprofiler-sdk-roctx.so.1", "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1", "libroctx64.so",
             "/opt/rocm/lib/libroctx64.so"]
    try:
        import torch
        cands.append(os.path.join(os.path.dirname(torch.__file__), "lib", "libroctx64.so"))
    except Exception:  # pragma: no cover
        pass
    for c in cands:
        try:
            lib = ctypes.CDLL(c)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            _state["lib"] = lib
            break
        except (OSError, AttributeError):
            continue
    return _state["lib"]


def tracing(enabled: bool | None = None) -> bool:
    """Turn the roctx ranges on / off (None: query); returns whether ranges are being emitted."""
    if enabled is not None:
        _state["enabled"] = bool(enabled)
    return _state["enabled"] and _load() is not None


@contextlib.contextmanager
def trace_range(name: str):
    lib = _load() if _state["enabled"] else None
    if lib is None:
        yield
        return
    lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        lib.roctxRangePop()
