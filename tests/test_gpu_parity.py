"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and sklearn's golden vectors.

Bar (north_star): W and H within 1e-5 relative Frobenius of the fp64 oracle run on IDENTICAL inputs
(the fp32 inputs promoted to fp64).  fp64 inputs: 1e-9.  bf16 X: the oracle runs on the
bf16-rounded values, same 1e-5 bar.  Iteration counts (tol > 0) must match exactly.
"""
import numpy as np
import pytest

from golden_io import load, names, rel_fro
from oracle import mu_ref

pytestmark = pytest.mark.gpu

TOL32 = 1e-5
TOL64 = 1e-9


def _api():
    import cnmf_amd
    return cnmf_amd


def _oracle_inputs(case):
    X = case["X"]
    kw = case["kwargs"]
    k = kw["n_components"]
    regs = mu_ref.compute_regularization(X.shape[0], X.shape[1], kw.get("alpha_W", 0.0),
                                         kw.get("alpha_H", "same"), kw.get("l1_ratio", 0.0))
    update_H = kw.get("update_H", True)
    if not update_H:
        W0, H0 = mu_ref.transform_init(X, k), case["H0"]
    elif kw["init"] == "random":
        from cnmf_amd.synthetic import random_init
        W0, H0 = random_init(X, k, kw.get("random_state"))
    else:
        W0, H0 = case["W0"], case["H0"]
    return X, W0, H0, regs, update_H


@pytest.mark.parametrize("name", names())
def test_golden_case_through_api(name):
    cnmf_amd = _api()
    case = load(name)
    kw = dict(case["kwargs"])
    X = case["X"]
    W0 = case.get("W0")
    H0 = case.get("H0")
    W, H, n_iter = cnmf_amd.factorise(X, None if W0 is None else W0.copy(),
                                      None if H0 is None else H0.copy(), **kw)
    assert W.dtype == X.dtype and H.dtype == X.dtype
    assert n_iter == case["n_iter"]
    Xo, W0o, H0o, regs, update_H = _oracle_inputs(case)
    Wr, Hr, nr = mu_ref.mu_fit(Xo.astype(np.float64), W0o.astype(np.float64), H0o.astype(np.float64),
                               max_iter=kw["max_iter"], tol=kw["tol"], l1_reg_W=regs[0],
                               l1_reg_H=regs[1], l2_reg_W=regs[2], l2_reg_H=regs[3],
                               update_H=update_H)
    tol = TOL64 if X.dtype == np.float64 else TOL32
    ew, eh = rel_fro(W, Wr), rel_fro(H, Hr)
    assert ew <= tol and eh <= tol, (name, ew, eh)
    # and against sklearn's own outputs on the same inputs (fp32 sklearn drifts from fp64 itself:
    # the measured distance is printed, and recorded by tools/parity_report.py)
    ref_tol = TOL64 if X.dtype == np.float64 else 1.2e-5  # measured <= 9.0e-6 (sklearn fp32's own drift)
    esw, esh = rel_fro(W, case["W"]), rel_fro(H, case["H"])
    skw, skh = rel_fro(case["W"], Wr), rel_fro(case["H"], Hr)
    print(f"{name}: GPU vs fp64 oracle W {ew:.2e} H {eh:.2e}; GPU vs sklearn W {esw:.2e} H {esh:.2e}; "
          f"sklearn vs fp64 oracle W {skw:.2e} H {skh:.2e}")
    assert esw <= ref_tol and esh <= ref_tol


def test_single_pass_matches_numpy():
    """One fused pass: W update and the [WᵀX | WᵀW] partial sums vs NumPy fp64 (ragged N, k=5)."""
    import torch
    from cnmf_amd.solver import MUPlan
    from cnmf_amd import _lib
    rng = np.random.default_rng(3)
    N, F, k = 1000 + 37, 81, 5
    X = rng.random((N, F)).astype(np.float32)
    X[7] = 0.0
    W0 = rng.random((N, k)).astype(np.float32)
    H0 = rng.random((k, F)).astype(np.float32)
    plan = MUPlan(torch.from_numpy(X).cuda(), k)
    plan.set_W(torch.from_numpy(W0))
    plan.set_H(torch.from_numpy(H0))
    plan.sample_pass(_lib.PASS_UPDATE_W | _lib.PASS_ACCUMULATE)
    plan.reduce(plan.n_out, plan.AB)
    torch.cuda.synchronize()
    Xd, Wd, Hd = X.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64)
    Wref, _, _ = mu_ref.update_w(Xd, Wd.copy(), Hd)
    Wg = plan.W.cpu().numpy()
    assert rel_fro(Wg, Wref) < 1e-6
    AB = plan.AB.cpu().numpy().reshape(k, F + k)
    Wn = Wg.astype(np.float64)
    np.testing.assert_allclose(AB[:, :F], Wn.T @ Xd, rtol=2e-6)
    np.testing.assert_allclose(AB[:, F:], Wn.T @ Wn, rtol=2e-6)


def test_loss_pass_matches_numpy():
    import torch
    from cnmf_amd.solver import MUPlan
    rng = np.random.default_rng(4)
    N, F, k = 777, 81, 4
    X = rng.random((N, F)).astype(np.float32)
    W0 = rng.random((N, k)).astype(np.float32)
    H0 = rng.random((k, F)).astype(np.float32)
    plan = MUPlan(torch.from_numpy(X).cuda(), k)
    plan.set_W(torch.from_numpy(W0))
    plan.set_H(torch.from_numpy(H0))
    err = plan.frobenius_error()
    ref = mu_ref.frobenius_error(X.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64))
    assert abs(err - ref) / ref < 1e-6


@pytest.mark.parametrize("dt", ["float32", "float64"])
def test_mid_size_500_iters(dt):
    """1e5 x 81, k=4, 500 fixed iterations (cfg2's shape class at an oracle-friendly size)."""
    cnmf_amd = _api()
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(100_000, 81, seed=0, dtype=np.dtype(dt))
    W0, H0 = random_init(X, 4, 42)
    W, H, n = cnmf_amd.factorise(X, W0.copy(), H0.copy(), n_components=4, init="custom", tol=0.0,
                                 max_iter=500)
    Wr, Hr, _ = mu_ref.mu_fit(X.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                              max_iter=500, tol=0.0)
    tol = TOL32 if dt == "float32" else TOL64
    assert rel_fro(W, Wr) <= tol and rel_fro(H, Hr) <= tol, (rel_fro(W, Wr), rel_fro(H, Hr))


def test_k8_500_iters_fp32():
    cnmf_amd = _api()
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(50_000, 81, seed=2, dtype=np.float32)
    W0, H0 = random_init(X, 8, 42)
    W, H, _ = cnmf_amd.factorise(X, W0.copy(), H0.copy(), n_components=8, init="custom", tol=0.0,
                                 max_iter=500)
    Wr, Hr, _ = mu_ref.mu_fit(X.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                              max_iter=500, tol=0.0)
    assert rel_fro(W, Wr) <= TOL32 and rel_fro(H, Hr) <= TOL32, (rel_fro(W, Wr), rel_fro(H, Hr))


def test_bf16_input_matches_oracle_on_rounded_values():
    import torch
    cnmf_amd = _api()
    from cnmf_amd.synthetic import iop_spectra, random_init
    X32 = iop_spectra(20_000, 300, seed=2, dtype=np.float32)
    Xb = torch.from_numpy(X32).to(torch.bfloat16)
    Xr = Xb.float().numpy()  # the values bf16 actually holds
    W0, H0 = random_init(Xr, 16, 42)
    W, H, _ = cnmf_amd.factorise(Xb.cuda(), torch.from_numpy(W0).cuda(), torch.from_numpy(H0).cuda(),
                                 n_components=16, init="custom", tol=0.0, max_iter=50)
    Wr, Hr, _ = mu_ref.mu_fit(Xr.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                              max_iter=50, tol=0.0)
    assert rel_fro(W.cpu().numpy(), Wr) <= TOL32 and rel_fro(H.cpu().numpy(), Hr) <= TOL32


def test_full_size_properties():
    """cfg2 at full size (1e6 x 81, k=4): determinism, non-negativity, monotone objective."""
    import torch
    from cnmf_amd.solver import MUPlan, run_mu
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(1_000_000, 81, seed=0, dtype=np.float32)
    W0, H0 = random_init(X, 4, 42)
    Xd = torch.from_numpy(X).cuda()
    errs = []
    outs = []
    for rep in range(2):
        plan = MUPlan(Xd, 4)
        plan.set_W(torch.from_numpy(W0))
        plan.set_H(torch.from_numpy(H0))
        prev = plan.frobenius_error()
        for _ in range(5):
            run_mu(plan, max_iter=10, tol=0.0)
            e = plan.frobenius_error()
            assert e <= prev * (1 + 1e-7)
            prev = e
        errs.append(prev)
        outs.append((plan.W.clone(), plan.H64.clone()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert bool((outs[0][0] >= 0).all()) and bool((outs[0][1] >= 0).all())


@pytest.mark.parametrize("norm", ["l1", "l2", "max"])
@pytest.mark.parametrize("dt", ["float32", "float64"])
def test_normalise_projection(norm, dt):
    """§8 a6: unit-norm basis rows, scales folded into W (W·H unchanged), vs the oracle."""
    import torch
    from cnmf_amd.solver import MUPlan
    rng = np.random.default_rng(8)
    N, F, k = 3001, 81, 5
    X = rng.random((N, F)).astype(dt)
    W0 = rng.random((N, k)).astype(dt)
    H0 = (rng.random((k, F)) * 3).astype(dt)
    H0[2] = 0.0  # an all-zero basis row keeps scale 1
    plan = MUPlan(torch.from_numpy(X).cuda(), k)
    plan.set_W(torch.from_numpy(W0))
    plan.set_H(torch.from_numpy(H0))
    s = plan.normalise(norm).cpu().numpy()
    Wr, Hr, sr = mu_ref.normalise(W0, H0, norm)
    np.testing.assert_allclose(s, sr, rtol=1e-14)
    W, H = plan.W.cpu().numpy(), plan.H64.cpu().numpy()
    assert rel_fro(H, Hr) < 1e-15
    assert rel_fro(W, Wr) < (1e-7 if dt == "float32" else 1e-15)
    np.testing.assert_allclose(plan.HHt.cpu().numpy()[:k, :k], H @ H.T, rtol=1e-13, atol=1e-15)
    err = plan.frobenius_error()  # Ht/HHt are consistent with the new H: the loss is unchanged
    ref = mu_ref.frobenius_error(X.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64))
    assert abs(err - ref) / ref < 1e-6


def test_factorise_normalise_option():
    cnmf_amd = _api()
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(20_000, 81, seed=1, dtype=np.float32)
    W0, H0 = random_init(X, 4, 42)
    W, H, n = cnmf_amd.factorise(X, W0.copy(), H0.copy(), n_components=4, init="custom", tol=0.0,
                                 max_iter=100, normalise="l2")
    Wr, Hr, _ = mu_ref.mu_fit(X.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                              max_iter=100, tol=0.0)
    Wn, Hn, _ = mu_ref.normalise(Wr, Hr, "l2")
    assert rel_fro(W, Wn) <= TOL32 and rel_fro(H, Hn) <= TOL32
    np.testing.assert_allclose(np.linalg.norm(H.astype(np.float64), axis=1), 1.0, rtol=1e-6)


@pytest.mark.parametrize("N, F, k", [(4096 + 29, 300, 16), (1000, 64, 12), (777, 300, 9), (3000, 124, 16),
                                     (64 * 700, 300, 16), (40, 300, 16), (64 * 1000 + 16, 320, 13),
                                     # the wave-tile slot's X row stride (§3.4): 2F already at the
                                     # stride (F = 48: no pad), the widest pad (F = 52: 56 B), k < 16
                                     (64 * 50 + 7, 48, 16), (64 * 30, 52, 16), (64 * 40 + 33, 96, 11)])
def test_bf16_mfma_single_pass_matches_numpy(N, F, k):
    """§8 a8: the bf16 matrix-core pass (the wave-tile mu_pass_bfw_kernel over the full 64-sample
    tiles, the 64-sample mu_pass_bf16_mfma_kernel on a ragged tail: v_mfma_f32_16x16x32 /
    16x16x16 bf16 with 3-term bf16 splits of H and (64-sample kernel) W' — two terms of W' in the
    wave-tile pass since round 5 — ds_read_b64_tr_b16 column reads): one W
    update and [WᵀX | WᵀW] vs NumPy fp64 on the bf16-rounded X (ragged last tile, no full tile at
    all, whole tiles only, k < 16 padding, F = 320, padded and unpadded LDS rows)."""
    import torch
    from cnmf_amd.solver import MUPlan
    from cnmf_amd import _lib
    rng = np.random.default_rng(N + F + k)
    Xb = torch.from_numpy(rng.random((N, F)).astype(np.float32)).to(torch.bfloat16)
    Xr = Xb.float().numpy().astype(np.float64)
    W0 = rng.random((N, k)).astype(np.float32)
    H0 = rng.random((k, F)).astype(np.float32)
    plan = MUPlan(Xb.cuda(), k)
    plan.set_W(torch.from_numpy(W0))
    plan.set_H(torch.from_numpy(H0))
    plan.sample_pass(_lib.PASS_UPDATE_W | _lib.PASS_ACCUMULATE)
    plan.reduce(plan.n_out, plan.AB)
    torch.cuda.synchronize()
    Wref, _, _ = mu_ref.update_w(Xr, W0.astype(np.float64), H0.astype(np.float64))
    Wg = plan.W.cpu().numpy()
    assert rel_fro(Wg, Wref) < 1e-6, rel_fro(Wg, Wref)
    AB = plan.AB.cpu().numpy().reshape(k, F + k)
    Wn = Wg.astype(np.float64)
    np.testing.assert_allclose(AB[:, :F], Wn.T @ Xr, rtol=2e-6)
    np.testing.assert_allclose(AB[:, F:], Wn.T @ Wn, rtol=2e-6)


@pytest.mark.parametrize("k, F, dt", [(12, 100, "float32"), (16, 300, "bfloat16"), (9, 37, "float64")])
def test_split_basis_update_iterations(k, F, dt):
    """k = 9..16 (KP = 16): the basis update spread over H's 16-feature blocks
    (basis_update_split_kernel, with the cross-block HHᵀ sum by the last arriver) inside the
    per-iteration path; 40 iterations against the fp64 oracle (bf16: on the rounded X)."""
    import torch
    from cnmf_amd.solver import MUPlan
    from cnmf_amd.synthetic import iop_spectra, random_init
    X32 = iop_spectra(30_000, F, seed=k + F, dtype=np.float32)
    if dt == "bfloat16":
        Xt = torch.from_numpy(X32).to(torch.bfloat16)
    else:
        Xt = torch.from_numpy(X32.astype(dt))
    Xr = Xt.double().numpy()
    W0, H0 = random_init(Xr.astype(np.float32), k, 42)
    plan = MUPlan(Xt.cuda(), k)
    plan.set_W(torch.from_numpy(W0))
    plan.set_H(torch.from_numpy(H0))
    plan.iterate(40)
    torch.cuda.synchronize()
    Wr, Hr, _ = mu_ref.mu_fit(Xr, W0.astype(np.float64), H0.astype(np.float64), max_iter=40, tol=0.0)
    W, H = plan.W.cpu().numpy(), plan.H64.cpu().numpy()
    bar = 1e-9 if dt == "float64" else TOL32
    assert rel_fro(W, Wr) <= bar and rel_fro(H, Hr) <= bar, (rel_fro(W, Wr), rel_fro(H, Hr))
    Ht, HHt = plan.Ht.cpu().numpy(), plan.HHt.cpu().numpy()
    np.testing.assert_array_equal(Ht[:, :k], H.T)
    assert not Ht[:, k:].any() and not HHt[k:, :].any() and not HHt[:, k:].any()
    np.testing.assert_allclose(HHt[:k, :k], H @ H.T, rtol=1e-12)
    assert plan.counters_at_rest()
