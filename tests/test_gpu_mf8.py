"""k = 8 on the matrix cores (mu_iter_mf8_kernel): the persistent wave-tile launch
whose two products run on v_mfma_f32_16x16x4_f32 (layout 5) against the fp64
oracle (north-star bar 1e-5), against the VALU wave tiles (layout 4, the default: fp32 summation-order
agreement), bit-for-bit repeatable across split launches, W resident (LDS) and streamed, with the
regularised update.

Since round 6 layout 5 lives in the diagnostic library only (it lost to layout 4
on every box), so each case runs in a child process with CNMF_HIP_LIB = cnmf_amd/libcnmf_hip_diag.so
(one process per case, sequential: the library is chosen when the process first loads it)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from golden_io import rel_fro
from oracle import mu_ref

pytestmark = pytest.mark.gpu

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_DIAG = os.path.join(_ROOT, "cnmf_amd", "libcnmf_hip_diag.so")


def _in_diag(call: str):
    """Run `call` (an expression over this module, imported as m) in a child on the diagnostic library."""
    code = (f"import sys; sys.path[:0] = [{_ROOT!r}, {os.path.join(_ROOT, 'tests')!r}]; "
            f"import test_gpu_mf8 as m; {call}")
    r = subprocess.run([sys.executable, "-u", "-c", code], cwd=_ROOT, capture_output=True, text=True,
                       timeout=500, env=dict(os.environ, CNMF_HIP_LIB=_DIAG))
    print(r.stdout[-2000:])
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])


def test_product_library_refuses_layout_5():
    """The product library has no matrix-core k = 8 tiles: layout 5 is CNMF_ERR_ARG there."""
    import ctypes
    import torch
    from cnmf_amd import _lib
    if "diag" in _lib.lib_path():
        pytest.skip("CNMF_HIP_LIB points at the diagnostic library")
    lib = _lib.load()
    buf = ctypes.create_string_buffer(256)
    assert torch.cuda.is_available()
    assert lib.cnmf_persist_describe(1_250_000, 81, 8, _lib.F32, 5, buf, 256) < 0
    assert b"diagnostic build" in lib.cnmf_last_error()


def _plan(X, W0, H0, layout=5, **regs):
    import torch
    from cnmf_amd.solver import MUPlan
    plan = MUPlan(torch.from_numpy(X).cuda(), W0.shape[1], **regs)
    plan.layout = layout
    plan.set_W(torch.from_numpy(W0))
    plan.set_H(torch.from_numpy(H0))
    return plan


@pytest.mark.timeout(600)
@pytest.mark.parametrize("n,iters", [(16 * 4000, 200), (1_250_000, 30)])
def test_mf8_matches_oracle_and_valu(n, iters):
    """64k rows: W resident in LDS; 1.25e6 rows (cfg3's shard): W streamed with X."""
    _in_diag(f"m.case_matches_oracle_and_valu({n}, {iters})")


def case_matches_oracle_and_valu(n, iters):
    import torch
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(n, 81, seed=n % 1009, dtype=np.float32)
    W0, H0 = random_init(X, 8, 42)
    a = _plan(X, W0, H0)
    assert a.persistent and "mu_iter_mf8_kernel" in a.describe(), a.describe()
    a.iterate(iters)
    a.check_sync_error()
    assert a.counters_at_rest()
    v = _plan(X, W0, H0, layout=0)
    assert "mu_iter_wt_kernel" in v.describe()
    v.iterate(iters)
    v.check_sync_error()
    Wa, Ha = a.W.cpu().numpy(), a.H64.cpu().numpy()
    assert rel_fro(Wa, v.W.cpu().numpy()) < 1e-6 and rel_fro(Ha, v.H64.cpu().numpy()) < 1e-6
    Wr, Hr, _ = mu_ref.mu_fit(X.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                              max_iter=iters, tol=0.0)
    assert rel_fro(Wa, Wr) <= 1e-5 and rel_fro(Ha, Hr) <= 1e-5, (rel_fro(Wa, Wr), rel_fro(Ha, Hr))
    np.testing.assert_array_equal(a.Ht.cpu().numpy()[:, :8], Ha.T)
    # split launches continue bit for bit
    c = _plan(X, W0, H0)
    for m in (1, iters // 3, iters - iters // 3 - 1):
        c.iterate(m)
    assert torch.equal(a.W, c.W) and torch.equal(a.H64, c.H64)


@pytest.mark.timeout(600)
def test_mf8_500_iterations_and_regularised():
    _in_diag("m.case_500_iterations_and_regularised()")


def case_500_iterations_and_regularised():
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(16 * 3125, 81, seed=2, dtype=np.float32)
    W0, H0 = random_init(X, 8, 42)
    a = _plan(X, W0, H0)
    a.iterate(500)
    Wr, Hr, _ = mu_ref.mu_fit(X.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                              max_iter=500, tol=0.0)
    ew, eh = rel_fro(a.W.cpu().numpy(), Wr), rel_fro(a.H64.cpu().numpy(), Hr)
    print(f"mf8 k8 50000 x 81, 500 it: rel W {ew:.2e} H {eh:.2e}")
    assert ew <= 1e-5 and eh <= 1e-5, (ew, eh)
    l1W, l2W, l1H, l2H = 0.05, 0.02, 0.1, 0.03
    r = _plan(X, W0, H0, l1_W=l1W, l2_W=l2W, l1_H=l1H, l2_H=l2H)
    r.iterate(100)
    Wr, Hr, _ = mu_ref.mu_fit(X.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                              max_iter=100, tol=0.0, l1_reg_W=l1W, l1_reg_H=l1H, l2_reg_W=l2W, l2_reg_H=l2H)
    assert rel_fro(r.W.cpu().numpy(), Wr) <= 1e-5 and rel_fro(r.H64.cpu().numpy(), Hr) <= 1e-5
