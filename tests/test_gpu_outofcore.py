"""Out-of-core MU (cnmf_amd/outofcore.py): X in host memory, streamed through
HBM in row chunks every iteration.

* The streaming schedule (copies on their own stream, n_buffers chunks in flight, buffers reused
  after an event) must not change a bit: a plan with 2 buffers over 4 chunks gives the same W and H
  as the same chunking loaded once (4 buffers, no per-iteration copies) — torch.equal, for X
  page-locked in place and for X staged through pinned buffers.
* Against the fp64 oracle (oracle/mu_ref.py, SK:526-728) at the north_star bar 1e-5, through the
  API with a memory budget below X's size, including a tol > 0 run whose n_iter must be sklearn's
  and a read-only memory-mapped .npy (staged copies).
"""
import numpy as np
import pytest

from golden_io import rel_fro
from oracle import mu_ref

pytestmark = pytest.mark.gpu

TOL32 = 1e-5


def _data(N, k=4, seed=0, dtype=np.float32):
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(N, 81, seed=seed, dtype=dtype)
    W0, H0 = random_init(X, k, 42)
    return X, W0, H0


def _splan(X, W0, H0, **kw):
    import torch
    from cnmf_amd.outofcore import StreamedMUPlan
    p = StreamedMUPlan(X, W0.shape[1], **kw)
    p.set_W(torch.from_numpy(W0))
    p.set_H(torch.from_numpy(H0))
    return p


@pytest.mark.parametrize("register", [True, False], ids=["registered", "staged"])
def test_streaming_is_bit_identical_to_resident_chunks(register):
    import torch
    X, W0, H0 = _data(64 * 3000 + 37, seed=1)
    s = _splan(X, W0, H0, chunk_rows=64 * 1000, n_buffers=2, register=register)
    r = _splan(X, W0, H0, chunk_rows=64 * 1000, n_buffers=4)
    assert s.n_chunks == 4 and s.mode == ("registered" if register else "staged") and r.mode == "resident"
    s.iterate(30)
    r.iterate(30)
    torch.cuda.synchronize()
    assert torch.equal(s.W, r.W) and torch.equal(s.H64, r.H64)
    assert s.frobenius_error() == r.frobenius_error()
    assert s.counters_at_rest()
    Wr, Hr, _ = mu_ref.mu_fit(X.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                              max_iter=30, tol=0.0)
    W, H = s.W.cpu().numpy(), s.H64.cpu().numpy()
    assert rel_fro(W, Wr) <= TOL32 and rel_fro(H, Hr) <= TOL32, (rel_fro(W, Wr), rel_fro(H, Hr))
    s.release()


def test_streamed_agrees_with_in_hbm_plan_k8():
    import torch
    from cnmf_amd.solver import MUPlan
    X, W0, H0 = _data(64 * 4000, k=8, seed=2)
    s = _splan(X, W0, H0, chunk_rows=64 * 1200, n_buffers=2)
    m = MUPlan(torch.from_numpy(X).cuda(), 8)
    m.set_W(torch.from_numpy(W0))
    m.set_H(torch.from_numpy(H0))
    s.iterate(40)
    m.iterate(40)
    m.check_sync_error()
    assert rel_fro(s.W.cpu().numpy(), m.W.cpu().numpy()) < 1e-6
    assert rel_fro(s.H64.cpu().numpy(), m.H64.cpu().numpy()) < 1e-6
    assert abs(s.frobenius_error() - m.frobenius_error()) <= 1e-7 * m.frobenius_error()


def test_api_memory_budget_tol_matches_oracle():
    import cnmf_amd
    X, W0, H0 = _data(64 * 2500 + 11, seed=3)
    W, H, n = cnmf_amd.factorise(X, W0.copy(), H0.copy(), n_components=4, init="custom", tol=1e-4,
                                 max_iter=300, memory_budget=X.nbytes // 3)
    Wr, Hr, nr = mu_ref.mu_fit(X.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                               max_iter=300, tol=1e-4)
    assert n == nr
    assert rel_fro(W, Wr) <= TOL32 and rel_fro(H, Hr) <= TOL32, (rel_fro(W, Wr), rel_fro(H, Hr))


def test_memory_mapped_npy_streams_staged(tmp_path):
    import cnmf_amd
    from cnmf_amd.outofcore import StreamedMUPlan
    X, W0, H0 = _data(64 * 1500, seed=4)
    path = tmp_path / "cube.npy"
    np.save(path, X)
    Xm = np.load(path, mmap_mode="r")
    p = StreamedMUPlan(Xm, 4, chunk_rows=64 * 400)
    assert p.mode == "staged" and p.n_chunks == 4  # read-only mapping: not page-locked in place
    est = cnmf_amd.NMF(4, init="custom", max_iter=50, tol=0.0, memory_budget=Xm.nbytes // 4)
    W = est.fit_transform(Xm, W=W0.copy(), H=H0.copy())
    Wr, Hr, _ = mu_ref.mu_fit(X.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                              max_iter=50, tol=0.0)
    assert rel_fro(W, Wr) <= TOL32 and rel_fro(est.components_, Hr) <= TOL32
    # transform (update_H=False) streams too
    Wt = est.transform(Xm)
    Wt_ref = mu_ref.mu_fit(X.astype(np.float64), np.full((X.shape[0], 4), np.sqrt(X.mean() / 4)),
                           est.components_.astype(np.float64), max_iter=50, tol=0.0, update_H=False)[0]
    assert rel_fro(Wt, Wt_ref) <= TOL32
