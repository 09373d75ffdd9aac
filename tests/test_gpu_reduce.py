"""GPU: cnmf_reduce_partials (include/cnmf_hip.h) against a NumPy fp64 column sum.

Wide rows (n_out >= 1024, <= 1024 partial rows) take the one-level reduce_wide_kernel since round 6
(cfg4's [WᵀX | WᵀW] rows, the init Gram rows); narrower or taller inputs keep the two-level
reduce_kernel.  Both sum in a fixed order: two runs are bit-identical.  Bar: 1e-13 relative to the
column's absolute sum (fp64 rounding of <= 1024 terms).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n_parts,n_out", [(0, 5056), (1, 5056), (7, 1024), (256, 5056), (257, 6642),
                                           (1024, 2000), (1100, 5056), (256, 340)])
def test_reduce_partials_matches_numpy(n_parts, n_out):
    import torch
    from cnmf_amd._lib import check, load

    def _ptr(t):
        return t.data_ptr()
    lib = load()
    dev = torch.device("cuda")
    rng = np.random.default_rng(n_parts * 7919 + n_out)
    P = rng.standard_normal((max(n_parts, 1), n_out)) * rng.uniform(0.5, 2e3, size=(1, n_out))
    parts = torch.from_numpy(P).to(dev)
    stage = torch.zeros(int(lib.cnmf_stage_doubles(n_out)), dtype=torch.float64, device=dev)
    counter = torch.zeros(int(lib.cnmf_counter_words()), dtype=torch.int32, device=dev)
    outs = []
    for _ in range(2):
        out = torch.full((n_out,), np.nan, dtype=torch.float64, device=dev)
        check(lib.cnmf_reduce_partials(_ptr(parts), n_parts, n_out, _ptr(stage), _ptr(counter), _ptr(out),
                                       torch.cuda.current_stream().cuda_stream), "cnmf_reduce_partials")
        torch.cuda.synchronize()
        outs.append(out.cpu().numpy())
    ref = P[:n_parts].sum(axis=0) if n_parts else np.zeros(n_out)
    scale = np.abs(P[:n_parts]).sum(axis=0) if n_parts else np.ones(n_out)
    assert np.all(np.abs(outs[0] - ref) <= 1e-13 * scale + 1e-300)
    assert np.array_equal(outs[0], outs[1])
    assert int(counter.abs().sum()) == 0  # tickets back at rest
