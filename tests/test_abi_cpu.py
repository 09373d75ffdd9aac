"""CPU-side checks of the C ABI: the library loads and exports every declared symbol; host-only
helpers answer without a GPU; the error path is a status code + message, never a crash."""
import pytest

from cnmf_amd import _lib


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    declared = _lib.declared_symbols()
    assert len(declared) >= 10
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, missing


def test_host_helpers():
    lib = _lib.load()
    assert lib.cnmf_abi_version() >= 100
    assert [lib.cnmf_padded_k(k) for k in (1, 4, 5, 8, 9, 16)] == [4, 4, 8, 8, 16, 16]
    assert lib.cnmf_padded_k(17) < 0 and lib.cnmf_padded_k(0) < 0
    assert lib.cnmf_stage_doubles(340) == 64 * 340


def test_error_paths_return_status():
    lib = _lib.load()
    st = lib.cnmf_mu_sample_pass(None, 0, None, None, None, None, 10, 81, 4, 0.0, 0.0, 3, None)
    assert st == -1
    assert b"null" in lib.cnmf_last_error()
    assert lib.cnmf_pass_blocks(100, 81, 17, 0) == -3  # k > 16 unsupported
    assert lib.cnmf_pass_blocks(100, 81, 4, 9) == -1   # unknown dtype
    with pytest.raises(_lib.HipLibraryError):
        _lib.check(-3, "probe")
    # a bad layout is refused before anything touches a device
    assert lib.cnmf_persist_describe(1024, 81, 4, 0, 7, b"\0" * 64, 64) == -1
    assert b"layout" in lib.cnmf_last_error()
    # the round-1 layouts 1-3 are in the diagnostic build only (VERDICT r3 housekeeping)
    for v in (1, 2, 3):
        assert lib.cnmf_persist_describe(1024, 81, 4, 0, v, b"\0" * 64, 64) == -1
        assert b"diagnostic" in lib.cnmf_last_error()
    assert lib.cnmf_abi_version() == 302


def test_product_library_has_no_diagnostic_switches():
    """the probe and the process-wide layout setters live in the diagnostic build."""
    lib = _lib.load()
    for name in ("cnmf_hbm_probe", "cnmf_set_persist_variant", "cnmf_get_persist_variant",
                 "cnmf_set_persist_dyn_frac"):
        assert not hasattr(lib, name), name


def test_prepared_calls_match_the_declared_signatures():
    """plan.prepare marshals each one-launch entry's arguments once (solver._prepared_call); the
    tuples it builds must match the ctypes signatures (checked here without a GPU call)."""
    import ctypes
    from cnmf_amd import _lib
    from cnmf_amd.solver import _prepared_call
    lib = _lib.load()
    ev = ((ctypes.c_void_p * 2)(1, 2), 2)
    calls = {
        "cnmf_mu_iterations": (20, 1, 0, 1, 1, 1, 1, 1, 8, 1, 1, 1, None, 1024, 81, 4, 0.0, 0.0, 0.0, 0.0, 0, *ev, 0),
        "cnmf_mu_iterations_multi": (20, 1, 0, 1, 1, 1, 1, 1, 8, 1, 1, 1, 1024, 81, 4, 0.0, 0.0, 0.0, 0.0, 1, 0, *ev,
                                     0),
        "cnmf_als_iterations": (20, 1, 0, 1, 1, 1, 1, 1, 1, 8, 1, 1, 1, 1024, 81, 4, 1.0, 0.5, *ev, 0),
        "cnmf_als_iterations_multi": (20, 1, 0, 1, 1, 1, 1, 1, 1, 8, 1, 1, 1, 1024, 81, 4, 1.0, 0.5, 1, *ev, 0),
        "cnmf_wmu_iterations": (20, 1, 1, 1, 1, 1, 8, 1, 1, 1, 1024, 81, 4, *ev, 0),
        "cnmf_wmu_iterations_multi": (20, 1, 1, 1, 1, 1, 8, 1, 1, 1, 1024, 81, 4, 1, *ev, 0),
    }
    import torch
    for name, args in calls.items():
        run = _prepared_call(getattr(lib, name), name, args, torch.device("cpu"))
        assert callable(run)
