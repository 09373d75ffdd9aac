"""GPU tests of the multi-GPU iteration (cnmf_mu_shard_step + all_reduce of [WᵀX | WᵀW]).

* one process: the shard-step sequence on the whole matrix reproduces the single-GPU launch;
* two processes sharing cuda:0 over gloo (RCCL needs distinct devices; the kernels and the host
  orchestration are the same): row shards reproduce the unsharded fp64 oracle within 1e-5.
"""
import os
import socket

import numpy as np
import pytest

from golden_io import rel_fro
from oracle import mu_ref

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("N", [64 * 2000, 50_000 + 17])
def test_shard_steps_match_single_gpu(N):
    import torch
    from cnmf_amd.solver import MUPlan
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(N, 81, seed=3, dtype=np.float32)
    W0, H0 = random_init(X, 4, 1)
    Xd = torch.from_numpy(X).cuda()
    a = MUPlan(Xd, 4)
    b = MUPlan(Xd, 4)
    for p in (a, b):
        p.set_W(torch.from_numpy(W0))
        p.set_H(torch.from_numpy(H0))
    a.iterate(30)
    for i in range(30):
        b.shard_step(apply_first=i > 0)
    b.basis_update()
    torch.cuda.synchronize()
    assert rel_fro(a.W.cpu().numpy(), b.W.cpu().numpy()) < 1e-6
    assert rel_fro(a.H64.cpu().numpy(), b.H64.cpu().numpy()) < 1e-6


def _worker(rank, world, port, X, W0, H0, n_iter, q, tol=1e-4):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cnmf_amd.distributed import shard_bounds
        from cnmf_amd.solver import MUPlan, run_mu
        lo, hi = shard_bounds(X.shape[0], world, rank)
        plan = MUPlan(torch.from_numpy(X[lo:hi]).cuda(), 4, group=dist.group.WORLD)
        assert plan.world == world
        plan.set_W(torch.from_numpy(W0[lo:hi]))
        plan.set_H(torch.from_numpy(H0))
        n = run_mu(plan, max_iter=n_iter, tol=tol)
        q.put((rank, lo, hi, plan.W.cpu().numpy(), plan.H64.cpu().numpy(), n))
    finally:
        dist.destroy_process_group()


def test_two_process_shards_match_oracle():
    import torch.multiprocessing as mp
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(64 * 1500, 81, seed=4, dtype=np.float32)
    W0, H0 = random_init(X, 4, 42)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, X, W0, H0, 200, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in procs]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    res.sort()
    W = np.concatenate([r[3] for r in res])
    H = res[0][4]
    assert np.array_equal(res[0][4], res[1][4])  # every rank applies the identical basis update
    assert res[0][5] == res[1][5]
    Wr, Hr, nr = mu_ref.mu_fit(X.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                               max_iter=200, tol=1e-4)
    assert res[0][5] == nr
    assert rel_fro(W, Wr) <= 1e-5 and rel_fro(H, Hr) <= 1e-5, (rel_fro(W, Wr), rel_fro(H, Hr))


def test_two_process_with_an_empty_shard():
    """world > rows: rank 1 owns no row; its shard contributes zeros to every all_reduce
    and still applies the identical basis update."""
    import torch.multiprocessing as mp
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(1, 81, seed=6, dtype=np.float32)
    W0, H0 = random_init(X, 4, 42)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, X, W0, H0, 60, q, 1e-3)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=100) for _ in procs)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert res[1][1] == res[1][2]  # rank 1's shard is empty
    assert np.array_equal(res[0][4], res[1][4]) and res[0][5] == res[1][5]
    Wr, Hr, nr = mu_ref.mu_fit(X.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                               max_iter=60, tol=1e-3)
    assert res[0][5] == nr
    assert rel_fro(res[0][3], Wr) <= 1e-5 and rel_fro(res[0][4], Hr) <= 1e-5


def _wworker(rank, world, port, X, M, W0, H0, n_iter, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cnmf_amd.distributed import factorise_sharded, shard_bounds
        lo, hi = shard_bounds(X.shape[0], world, rank)
        W, H, n = factorise_sharded(torch.from_numpy(X[lo:hi]), W0[lo:hi], H0, max_iter=n_iter,
                                    tol=1e-3, weights=M[lo:hi])
        q.put((rank, lo, hi, W.cpu().numpy(), H.double().cpu().numpy(), n))
    finally:
        dist.destroy_process_group()


def test_two_process_weighted_shards_match_oracle():
    """The weighted / masked MU sharded over 2 processes (factorise_sharded(weights=...))."""
    import torch.multiprocessing as mp
    from oracle import wmu_ref
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(3001, 81, seed=8, dtype=np.float32)
    rng = np.random.default_rng(8)
    M = (rng.uniform(0.2, 2.0, X.shape) * (rng.random(X.shape) >= 0.3)).astype(np.float32)
    W0, H0 = random_init(X, 4, 42)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_wworker, args=(r, 2, port, X, M, W0, H0, 200, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in procs]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    res.sort()
    W = np.concatenate([r[3] for r in res])
    H = res[0][4]
    assert np.array_equal(res[0][4], res[1][4]) and res[0][5] == res[1][5]
    Wr, Hr, nr = wmu_ref.wmu_fit(X.astype(np.float64), M.astype(np.float64), W0.astype(np.float64),
                                 H0.astype(np.float64), max_iter=200, tol=1e-3)
    assert res[0][5] == nr
    assert rel_fro(W, Wr) <= 1e-5 and rel_fro(H, Hr) <= 1e-5, (rel_fro(W, Wr), rel_fro(H, Hr))


def _sharded_als_worker(rank, world, port, X, W0, H0, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import warnings
        warnings.filterwarnings("error", message="in-launch exchange not used")  # no silent fallback
        torch.cuda.set_device(0)
        from cnmf_amd.distributed import factorise_sharded, shard_bounds
        lo, hi = shard_bounds(X.shape[0], world, rank, align=64)
        W, H, n = factorise_sharded(X[lo:hi], W0[lo:hi], H0, max_iter=25, tol=0.0, solver="als",
                                    sum_to_one=1.0, smoothness=0.5, exchange=True)
        q.put((rank, W.cpu().numpy(), H.cpu().numpy().astype(np.float64), n, None))
    except Exception as ex:  # reported to the parent
        q.put((rank, None, None, None, f"{type(ex).__name__}: {ex}"))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_factorise_sharded_als_exchange_matches_oracle():
    """The public sharded entry with solver='als' and exchange=True (the persistent ALS launch per rank
    with the all-reduce inside it), two processes on one GPU, against the fp64 ALS oracle."""
    import torch.multiprocessing as mp
    from oracle import als_ref
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(64 * 300, 81, seed=6, dtype=np.float32)
    W0, H0 = random_init(X, 4, 42)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_als_worker, args=(r, 2, port, X, W0, H0, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=300) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    errs = [r[4] for r in res if r[4]]
    assert not errs, errs
    assert np.array_equal(res[0][2], res[1][2])
    W = np.concatenate([r[1] for r in res])
    Wr, Hr, _ = als_ref.als_fit(X.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                                max_iter=25, tol=0.0, sum_to_one=1.0, smoothness=0.5)
    assert rel_fro(W, Wr) <= 1e-5 and rel_fro(res[0][2], Hr) <= 1e-5, (rel_fro(W, Wr), rel_fro(res[0][2], Hr))
