"""GPU parity of the weighted / masked MU (cnmf_wmu_sample_pass + reduction + cnmf_wmu_basis_update;
SURVEY.md §8(f) row 2) against the fp64 oracle (oracle/wmu_ref.py) on the same fp32 inputs.

Bar: 1e-5 relative Frobenius on W and H (north_star).  Shapes cover the tile sizes of the pass
(F = 81: 64-sample tiles; F = 300: 16-sample tiles and two features per thread in phase 2; F = 17
with k = 3), ragged row counts, masks with 30 % missing entries, unit weights against sklearn's
golden (cfg1), the tol stop through the API, and the weighted loss.
"""
import numpy as np
import pytest

from golden_io import load, rel_fro
from oracle import wmu_ref

pytestmark = pytest.mark.gpu

TOL32 = 1e-5


def _weights(X, seed, p_missing=0.3):
    rng = np.random.default_rng(seed)
    return (rng.uniform(0.2, 2.0, X.shape) * (rng.random(X.shape) >= p_missing)).astype(np.float32)


def _plan(X, M, W0, H0):
    import torch
    from cnmf_amd.solver import WeightedMUPlan
    plan = WeightedMUPlan(torch.from_numpy(X).cuda(), torch.from_numpy(M).cuda(), W0.shape[1])
    plan.set_W(torch.from_numpy(W0))
    plan.set_H(torch.from_numpy(H0))
    return plan


def test_unit_weights_match_sklearn_golden():
    case = load("cfg1_float32")
    X = case["X"]
    plan = _plan(X, np.ones_like(X), case["W0"], case["H0"])
    plan.iterate(200)
    W, H = plan.W.cpu().numpy(), plan.H64.cpu().numpy()
    Wr, Hr, _ = wmu_ref.wmu_fit(X.astype(np.float64), np.ones(X.shape), case["W0"].astype(np.float64),
                                case["H0"].astype(np.float64), max_iter=200, tol=0)
    assert rel_fro(W, Wr) <= TOL32 and rel_fro(H, Hr) <= TOL32, (rel_fro(W, Wr), rel_fro(H, Hr))
    # and sklearn's own fp32 run (its fp32 arithmetic differs in the last bits)
    assert rel_fro(W, case["W"]) <= 1e-4 and rel_fro(H, case["H"]) <= 1e-4


@pytest.mark.parametrize("n,F,k", [(5000, 81, 4), (4099, 81, 4), (3001, 300, 8), (777, 17, 3), (64, 81, 1)])
def test_masked_matches_oracle(n, F, k):
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(n, F, seed=n, dtype=np.float32)
    M = _weights(X, n)
    W0, H0 = random_init(X, k, 7)
    plan = _plan(X, M, W0, H0)
    n_it = 100
    plan.iterate(n_it)
    W, H = plan.W.cpu().numpy(), plan.H64.cpu().numpy()
    Wr, Hr, _ = wmu_ref.wmu_fit(X.astype(np.float64), M.astype(np.float64), W0.astype(np.float64),
                                H0.astype(np.float64), max_iter=n_it, tol=0)
    assert rel_fro(W, Wr) <= TOL32 and rel_fro(H, Hr) <= TOL32, (rel_fro(W, Wr), rel_fro(H, Hr))
    err = plan.frobenius_error()
    ref = wmu_ref.weighted_error(X.astype(np.float64), M.astype(np.float64), W.astype(np.float64), H)
    assert abs(err - ref) <= 1e-7 * ref  # the pass multiplies with the fp32-rounded basis


def test_tol_stop_through_api():
    import cnmf_amd
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(2000, 81, seed=4, dtype=np.float32)
    M = _weights(X, 4)
    W0, H0 = random_init(X, 4, 42)
    W, H, n = cnmf_amd.factorise(X, W0.copy(), H0.copy(), n_components=4, init="custom", tol=1e-3,
                                 max_iter=400, weights=M)
    Wr, Hr, nr = wmu_ref.wmu_fit(X.astype(np.float64), M.astype(np.float64), W0.astype(np.float64),
                                 H0.astype(np.float64), max_iter=400, tol=1e-3)
    assert n == nr
    assert rel_fro(W, Wr) <= TOL32 and rel_fro(H, Hr) <= TOL32
    est = cnmf_amd.NMF(4, init="custom", tol=1e-3, max_iter=400)
    W2 = est.fit_transform(X, W=W0.copy(), H=H0.copy(), weights=M)
    assert est.n_iter_ == nr and rel_fro(W2, Wr) <= TOL32
    assert abs(est.reconstruction_err_ - wmu_ref.weighted_error(
        X.astype(np.float64), M.astype(np.float64), W2.astype(np.float64),
        est.components_.astype(np.float64))) <= 1e-6 * est.reconstruction_err_


def test_native_library_used():
    """The weighted path is the HIP library's (no CPU fallback exists)."""
    from cnmf_amd import _lib
    lib = _lib.load()
    assert lib.cnmf_wmu_pass_blocks(1000, 81, 4) > 0
    assert lib.cnmf_wmu_pass_blocks(1000, 600, 4) < 0  # F > 512: refused, not emulated


def test_fully_masked_rows_and_columns():
    """A sample with every weight 0 (num = den = 0 -> eps: its w becomes 0) and a feature with every
    weight 0 (its H column becomes 0), as in the oracle; the rest still matches at 1e-5."""
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(1500, 81, seed=21, dtype=np.float32)
    M = _weights(X, 21)
    M[[0, 77, 1499], :] = 0.0
    M[:, [5, 80]] = 0.0
    W0, H0 = random_init(X, 4, 2)
    plan = _plan(X, M, W0, H0)
    plan.iterate(40)
    W, H = plan.W.cpu().numpy(), plan.H64.cpu().numpy()
    Wr, Hr, _ = wmu_ref.wmu_fit(X.astype(np.float64), M.astype(np.float64), W0.astype(np.float64),
                                H0.astype(np.float64), max_iter=40, tol=0)
    assert np.all(W[[0, 77, 1499]] == 0) and np.all(Wr[[0, 77, 1499]] == 0)
    assert np.all(H[:, [5, 80]] == 0) and np.all(Hr[:, [5, 80]] == 0)
    assert rel_fro(W, Wr) <= TOL32 and rel_fro(H, Hr) <= TOL32, (rel_fro(W, Wr), rel_fro(H, Hr))


# ---- the persistent weighted launch (wmu_iter_wt_kernel: fp32, F = 81, k = 4, rows % 16 == 0)

def _oracle_fit(X, M, W0, H0, n_it):
    return wmu_ref.wmu_fit(X.astype(np.float64), M.astype(np.float64), W0.astype(np.float64),
                           H0.astype(np.float64), max_iter=n_it, tol=0)


@pytest.mark.parametrize("n", [192 * 16, 5008, 65536])
def test_persistent_matches_oracle(n):
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(n, 81, seed=n, dtype=np.float32)
    M = _weights(X, n)
    W0, H0 = random_init(X, 4, 7)
    plan = _plan(X, M, W0, H0)
    assert plan.persistent, "fp32 F=81 k=4 rows % 16 == 0 takes the persistent weighted launch"
    n_it = 100
    plan.iterate(n_it)
    plan.check_sync_error()
    W, H = plan.W.cpu().numpy(), plan.H64.cpu().numpy()
    Wr, Hr, _ = _oracle_fit(X, M, W0, H0, n_it)
    assert rel_fro(W, Wr) <= TOL32 and rel_fro(H, Hr) <= TOL32, (rel_fro(W, Wr), rel_fro(H, Hr))
    assert int(plan.counter.abs().sum()) == 0  # tickets and flag left at rest


def test_persistent_split_launches_and_repeatable():
    """n iterations as one launch == as launches of 7 + 13 (the launch boundary carries W and H64
    only); two runs are bit-identical (no order depends on arrival); the per-iteration kernels
    agree at the fp32 rounding of their different summation orders."""
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(40000, 81, seed=3, dtype=np.float32)
    M = _weights(X, 3)
    W0, H0 = random_init(X, 4, 1)
    runs = []
    for split in ([20], [20], [7, 13]):
        plan = _plan(X, M, W0, H0)
        assert plan.persistent
        for n in split:
            plan.iterate(n)
        runs.append((plan.W.cpu().numpy(), plan.H64.cpu().numpy()))
    assert np.array_equal(runs[0][0], runs[1][0]) and np.array_equal(runs[0][1], runs[1][1])
    assert np.array_equal(runs[0][0], runs[2][0]) and np.array_equal(runs[0][1], runs[2][1])
    plan = _plan(X, M, W0, H0)
    plan.persistent = False  # the per-iteration pass + reduce + H-step launches
    plan.iterate(20)
    assert rel_fro(plan.W.cpu().numpy(), runs[0][0]) <= 1e-6
    assert rel_fro(plan.H64.cpu().numpy(), runs[0][1]) <= 1e-6


def test_persistent_fully_masked_rows_and_columns():
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(1504, 81, seed=21, dtype=np.float32)
    M = _weights(X, 21)
    M[[0, 77, 1503], :] = 0.0
    M[:, [5, 80]] = 0.0
    W0, H0 = random_init(X, 4, 2)
    plan = _plan(X, M, W0, H0)
    assert plan.persistent
    plan.iterate(40)
    W, H = plan.W.cpu().numpy(), plan.H64.cpu().numpy()
    Wr, Hr, _ = _oracle_fit(X, M, W0, H0, 40)
    assert np.all(W[[0, 77, 1503]] == 0) and np.all(H[:, [5, 80]] == 0)
    assert rel_fro(W, Wr) <= TOL32 and rel_fro(H, Hr) <= TOL32, (rel_fro(W, Wr), rel_fro(H, Hr))


def test_persistent_tol_stop_through_api():
    import cnmf_amd
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(4000, 81, seed=4, dtype=np.float32)
    M = _weights(X, 4)
    W0, H0 = random_init(X, 4, 42)
    W, H, n = cnmf_amd.factorise(X, W0.copy(), H0.copy(), n_components=4, init="custom", tol=1e-3,
                                 max_iter=400, weights=M)
    Wr, Hr, nr = wmu_ref.wmu_fit(X.astype(np.float64), M.astype(np.float64), W0.astype(np.float64),
                                 H0.astype(np.float64), max_iter=400, tol=1e-3)
    assert n == nr
    assert rel_fro(W, Wr) <= TOL32 and rel_fro(H, Hr) <= TOL32


def test_persistent_full_size():
    """The bench shape (1e6 x 81, k = 4, 30 % zero weights): 10 iterations against the fp64 oracle
    and the weighted error non-increasing over the launch boundaries."""
    import torch
    from cnmf_amd.synthetic import iop_spectra, random_init
    n = 1_000_000
    X = iop_spectra(n, 81, seed=0, dtype=np.float32)
    M = _weights(X, 0)
    W0, H0 = random_init(X, 4, 42)
    plan = _plan(X, M, W0, H0)
    assert plan.persistent
    errs = [plan.frobenius_error()]
    for _ in range(5):
        plan.iterate(2)
        plan.check_sync_error()
        errs.append(plan.frobenius_error())
    assert all(b <= a * (1 + 1e-12) for a, b in zip(errs, errs[1:])), errs
    W, H = plan.W.cpu().numpy(), plan.H64.cpu().numpy()
    assert np.all(np.isfinite(W)) and np.all(W >= 0) and np.all(H >= 0)
    del plan
    torch.cuda.empty_cache()
    Wr, Hr, _ = _oracle_fit(X, M, W0, H0, 10)
    assert rel_fro(W, Wr) <= TOL32 and rel_fro(H, Hr) <= TOL32, (rel_fro(W, Wr), rel_fro(H, Hr))


# ---- multi-GPU: the persistent weighted MU with the [A | D] all-reduce inside the launch

def _port():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _plan_group(X, M, W0, H0, group):
    import torch
    from cnmf_amd.solver import WeightedMUPlan
    plan = WeightedMUPlan(torch.from_numpy(X).cuda(), torch.from_numpy(M).cuda(), W0.shape[1], group=group)
    plan.set_W(torch.from_numpy(W0))
    plan.set_H(torch.from_numpy(H0))
    return plan


def _wdata(n, seed):
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(n, 81, seed=seed, dtype=np.float32)
    M = _weights(X, seed + 1)
    W0, H0 = random_init(X, 4, 42)
    return X, M, W0, H0


def test_persistent_self_exchange_is_bit_identical():
    """One rank exchanging with itself: bit-identical to the single-GPU launch, across launches."""
    import torch
    import torch.distributed as dist
    X, M, W0, H0 = _wdata(64 * 700, 3)
    ref = _plan(X, M, W0, H0)
    assert ref.persistent
    ref.iterate(15)
    ref.check_sync_error()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1)
    try:
        plan = _plan_group(X, M, W0, H0, dist.group.WORLD)
        plan.enable_exchange()
        assert plan.exchange and plan.persistent
        plan.iterate(6)
        plan.iterate(9)
        plan.check_sync_error()
        torch.cuda.synchronize()
        assert int(plan.xctl[3].item()) == 15
        assert torch.equal(plan.W, ref.W) and torch.equal(plan.H64, ref.H64)
        plan.release()
    finally:
        dist.destroy_process_group()


def _wmu_rank_main(rank, world, port, N, q):
    try:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        X, M, W0, H0 = _wdata(N, 5)
        lo, hi = rank * N // world, (rank + 1) * N // world
        plan = _plan_group(X[lo:hi].copy(), M[lo:hi].copy(), W0[lo:hi].copy(), H0, dist.group.WORLD)
        plan.enable_exchange()
        plan.iterate(11)
        plan.iterate(14)
        plan.check_sync_error()
        q.put((rank, plan.W.cpu().numpy(), plan.H64.cpu().numpy(), None))
        dist.barrier()
        plan.release()
        dist.destroy_process_group()
    except Exception as ex:  # reported to the parent
        q.put((rank, None, None, f"{type(ex).__name__}: {ex}"))


@pytest.mark.timeout(600)
def test_persistent_two_ranks_one_gpu_exchange():
    """Two processes on one GPU, half the rows each, exchanging [A | D] through IPC-mapped buffers
    inside the persistent weighted launch: the same H on both ranks, the fp64 oracle at 1e-5."""
    import multiprocessing as mp
    world, N = 2, 2 * 16 * 700
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_wmu_rank_main, args=(r, world, port, N, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            r, W, H, err = q.get(timeout=400)
            out[r] = (W, H, err)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    errs = [v[2] for v in out.values() if v[2]]
    assert not errs, errs
    np.testing.assert_array_equal(out[0][1], out[1][1])
    W = np.concatenate([out[0][0], out[1][0]])
    X, M, W0, H0 = _wdata(N, 5)
    Wr, Hr, _ = wmu_ref.wmu_fit(X.astype(np.float64), M.astype(np.float64), W0.astype(np.float64),
                                H0.astype(np.float64), max_iter=25, tol=0)
    assert rel_fro(W, Wr) <= TOL32 and rel_fro(out[0][1], Hr) <= TOL32, (rel_fro(W, Wr), rel_fro(out[0][1], Hr))
