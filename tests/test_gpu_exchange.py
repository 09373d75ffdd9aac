"""GPU tests of the in-launch cross-rank all-reduce (cnmf_mu_iterations_multi, MUPlan.enable_exchange).

On one MI355X the exchange is exercised two ways:
  * world 1: the rank exchanges with itself (its own buffer through the same system-scope stores,
    flags and loads); 0.0 + AB == AB, so the factors must be bit-identical to cnmf_mu_iterations,
    including across several launches (the generation counter carries over);
  * world 2 on the same GPU: two processes, each with a small shard (a 32-workgroup grid, so both
    persistent grids are resident at once), exchange through IPC-mapped fine-grained buffers; both
    ranks must end with the same H bit for bit and match the single-process run on the whole X to
    partial-sum-order noise (1e-6), and the oracle within the north_star bar.
The 8-GPU case (xGMI peers) runs only in the driver's scaling bench, which validates the exchange
against the RCCL path before timing it (bench.py).
"""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

from golden_io import rel_fro
from oracle import mu_ref

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _data(N, seed, k=4):
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(N, 81, seed=seed, dtype=np.float32)
    W0, H0 = random_init(X, k, 42)
    return X, W0, H0


def _plan(X, W0, H0, group=None, layout=0):
    import torch
    from cnmf_amd.solver import MUPlan
    plan = MUPlan(torch.from_numpy(X).cuda(), W0.shape[1], group=group)
    plan.layout = layout
    plan.set_W(torch.from_numpy(W0))
    plan.set_H(torch.from_numpy(H0))
    return plan


@pytest.fixture(params=[4], ids=["wave"])
def layout(request):
    """Every persistent layout a rank may pick at k = 4 in the product library (the wave tiles)."""
    return request.param


def test_self_exchange_is_bit_identical(layout):
    import torch
    import torch.distributed as dist
    from cnmf_amd import _lib
    X, W0, H0 = _data(64 * 1500, 5)
    ref = _plan(X, W0, H0, layout=layout)
    assert ref.persistent
    ref.iterate(25)
    ref.check_sync_error()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1)
    try:
        plan = _plan(X, W0, H0, group=dist.group.WORLD, layout=layout)
        plan.enable_exchange()
        assert plan.exchange and plan.persistent
        plan.iterate(10)
        plan.iterate(15)  # a second launch: generations 11..25
        plan.check_sync_error()
        assert int(plan.xctl[3].item()) == 25  # the device-side generation base
        torch.cuda.synchronize()
        assert torch.equal(plan.W, ref.W)
        assert torch.equal(plan.H64, ref.H64)
        assert torch.equal(plan.HHt, ref.HHt)
        assert plan.counters_at_rest()
        plan.release()
    finally:
        dist.destroy_process_group()


def _rank_main(rank, world, port, N, q, k=4):
    try:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                world_size=world)
        X, W0, H0 = _data(N, 7, k=k)
        lo, hi = rank * N // world, (rank + 1) * N // world
        plan = _plan(X[lo:hi].copy(), W0[lo:hi].copy(), H0, group=dist.group.WORLD)
        plan.enable_exchange()
        plan.iterate(12)
        plan.iterate(18)
        plan.check_sync_error()
        e = plan.frobenius_error()
        q.put((rank, plan.W.cpu().numpy(), plan.H64.cpu().numpy(), e, None))
        dist.barrier()
        plan.release()
        dist.destroy_process_group()
    except Exception as ex:  # reported to the parent
        q.put((rank, None, None, None, f"{type(ex).__name__}: {ex}"))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("k", [4, 8])
def test_two_ranks_one_gpu_exchange(k):
    """Two processes on one GPU exchanging through IPC-mapped buffers inside the persistent launch
    (k = 8: cfg3's shape, the wave-tile kernel's xchg_allreduce_n over 712 accumulators)."""
    import torch
    world, N = 2, 2 * 64 * 128  # 128 64-row tiles per rank
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    env_keep = os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY")
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, N, q, k)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            r, W, H, e, err = q.get(timeout=400)
            out[r] = (W, H, e, err)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    errs = [v[3] for v in out.values() if v[3]]
    assert not errs, errs
    assert env_keep in (None, "0")
    H0_, H1_ = out[0][1], out[1][1]
    np.testing.assert_array_equal(H0_, H1_)  # rank-ordered sums: the same H everywhere
    W = np.concatenate([out[0][0], out[1][0]])
    X, W0, H0 = _data(N, 7, k=k)
    ref = _plan(X, W0, H0)
    ref.iterate(30)
    ref.check_sync_error()
    torch.cuda.synchronize()
    # a different grid (per-rank grids of 32 workgroups vs one grid over all tiles) chains the
    # per-workgroup fp32 partial sums differently: ~1e-7 on AB, the same bar as the persistent vs
    # per-iteration-launch agreement (test_gpu_persistent.py)
    assert rel_fro(H0_, ref.H64.cpu().numpy()) < 1e-6
    assert rel_fro(W, ref.W.cpu().numpy()) < 1e-6
    Wr, Hr, _ = mu_ref.mu_fit(X.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                              max_iter=30, tol=0.0)
    assert rel_fro(W, Wr) <= 1e-5 and rel_fro(H0_, Hr) <= 1e-5
    assert abs(out[0][2] - out[1][2]) <= 1e-12 * out[0][2]  # the loss all-reduce agrees too


@pytest.mark.parametrize("N", [64 * 1500, 1_250_048])
def test_self_exchange_k8(N):
    """k = 8 (cfg3's shape) through the in-launch exchange with itself: the wave-tile kernel with W
    LDS-resident (96k rows) and streamed (a cfg3 shard), bit-identical to the single-GPU launch."""
    import torch
    import torch.distributed as dist
    X, W0, H0 = _data(N, 9, k=8)
    ref = _plan(X, W0, H0)
    assert ref.persistent
    ref.iterate(14)
    ref.check_sync_error()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1)
    try:
        plan = _plan(X, W0, H0, group=dist.group.WORLD)
        plan.enable_exchange()
        assert plan.exchange and plan.persistent
        plan.iterate(5)
        plan.iterate(9)
        plan.check_sync_error()
        torch.cuda.synchronize()
        assert torch.equal(plan.W, ref.W)
        assert torch.equal(plan.H64, ref.H64)
        assert plan.counters_at_rest()
        plan.release()
    finally:
        dist.destroy_process_group()


def _wide_rank_main(rank, world, port, rows, q):
    """One rank of the world-4 / world-8 exchange test: 12 + 18 iterations as two launches, then a
    second plan (fresh buffers) running the 30 as one launch."""
    try:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                world_size=world)
        X, W0, H0 = _data(world * rows, 7)
        lo, hi = rank * rows, (rank + 1) * rows
        outs = []
        for split in ((12, 18), (30,)):
            plan = _plan(X[lo:hi].copy(), W0[lo:hi].copy(), H0, group=dist.group.WORLD)
            g = int(plan.lib.cnmf_persist_workgroups(plan.n_rows, 81, 4, 0, 0, 1))
            plan.enable_exchange()
            for n in split:
                plan.iterate(n)
            plan.check_sync_error()
            torch.cuda.synchronize()
            outs.append((plan.W.cpu().numpy(), plan.H64.cpu().numpy(), int(plan.xctl[3].item())))
            assert plan.counters_at_rest()
            dist.barrier()
            plan.release()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, outs, g, None))
    except Exception as ex:  # reported to the parent
        q.put((rank, None, None, f"{type(ex).__name__}: {ex}"))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [4, 8])
def test_wide_world_one_gpu_exchange(world):
    """the in-launch exchange (cnmf_mu_iterations_multi) at world 4 and 8 before
    the driver's 8-GPU node meets it — `world` processes on one GPU, each rank's grid capped by its
    shard (4096 rows = 256 tiles = 16 workgroups per rank; 64-128 of the 256 CUs in all, so every
    rank's persistent grid is co-resident) exchanging through IPC-mapped buffers with the slot-per-rank
    generation / parity protocol.  Every rank must hold the same H bit for bit; W / H agree with the
    single-process run on the whole X to summation-order noise and with the fp64 oracle at 1e-5; two
    launches (12 + 18) equal one (30) bit for bit on every rank, and the device-side generation base
    advanced by 30 on every rank."""
    import torch
    rows = 4096
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_wide_rank_main, args=(r, world, port, rows, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            r, outs, g, err = q.get(timeout=500)
            out[r] = (outs, g, err)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    errs = [v[2] for v in out.values() if v[2]]
    assert not errs, errs
    assert sorted(out) == list(range(world))
    grids = [out[r][1] for r in range(world)]
    assert sum(grids) <= 256 and min(grids) >= 1, grids
    H = out[0][0][0][1]
    for r in range(world):
        (Wa, Ha, gena), (Wb, Hb, genb) = out[r][0]
        np.testing.assert_array_equal(Ha, H)  # rank-ordered sums: the same H on every rank
        np.testing.assert_array_equal(Hb, Ha)  # split launches == one launch, bit for bit
        np.testing.assert_array_equal(Wb, Wa)
        assert gena == genb == 30
    W = np.concatenate([out[r][0][0][0] for r in range(world)])
    X, W0, H0 = _data(world * rows, 7)
    ref = _plan(X, W0, H0)
    ref.iterate(30)
    ref.check_sync_error()
    torch.cuda.synchronize()
    assert rel_fro(H, ref.H64.cpu().numpy()) < 1e-6
    assert rel_fro(W, ref.W.cpu().numpy()) < 1e-6
    Wr, Hr, _ = mu_ref.mu_fit(X.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                              max_iter=30, tol=0.0)
    print(f"world {world}: grids {grids}; vs oracle W {rel_fro(W, Wr):.2e} H {rel_fro(H, Hr):.2e}")
    assert rel_fro(W, Wr) <= 1e-5 and rel_fro(H, Hr) <= 1e-5
