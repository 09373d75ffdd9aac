"""Host logic of the out-of-core fit (cnmf_amd/outofcore.py): chunk planning and
the API's decision to stream (no GPU needed)."""
import numpy as np
import pytest


def test_chunk_bounds_cover_rows_once():
    from cnmf_amd.outofcore import chunk_bounds
    for n, c in [(1, 64), (64, 64), (65, 64), (192037, 64000), (10 ** 6, 1 << 18)]:
        b = chunk_bounds(n, c)
        assert b[0][0] == 0 and b[-1][1] == n
        assert all(hi0 == lo1 for (_, hi0), (lo1, _) in zip(b, b[1:]))
        assert all(hi - lo == c for lo, hi in b[:-1]) and 0 < b[-1][1] - b[-1][0] <= c
    with pytest.raises(ValueError):
        chunk_bounds(10, 0)


def test_chunk_rows_for_budget():
    from cnmf_amd.outofcore import chunk_rows_for_budget
    r = chunk_rows_for_budget(1 << 30, 81, 4, 2)
    assert r % 64 == 0 and 2 * r * 81 * 4 <= 1 << 30 and 2 * (r + 64) * 81 * 4 > 1 << 30
    assert chunk_rows_for_budget(100, 81, 4) == 64  # never below one tile


def test_streaming_decision():
    from cnmf_amd.api import _streamed
    X = np.ones((1000, 81), np.float32)
    assert not _streamed(X, False, None, "mu", None)
    assert not _streamed(X, False, X.nbytes, "mu", None)  # fits the budget: in HBM
    assert _streamed(X, False, X.nbytes - 1, "mu", None)
    with pytest.raises(ValueError):
        _streamed(X, False, 1000, "als", None)
    with pytest.raises(ValueError):
        _streamed(X, False, 1000, "mu", np.ones_like(X))
    with pytest.raises(ValueError):
        _streamed(X, False, -5, "mu", None)


def test_memory_budget_is_an_estimator_param():
    import cnmf_amd
    est = cnmf_amd.NMF(4, memory_budget=1 << 30)
    assert est.get_params()["memory_budget"] == 1 << 30
