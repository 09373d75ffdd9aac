"""The device tolerance test inside the multi-GPU launch: `factorise_sharded`
with tol > 0 on wave-tile shards and the in-launch exchange enabled runs the whole fit as ONE
launch per rank of the exchange-plus-tolerance kernel (mu_iter_wt_kernel<…, MULTI, TOL>): the
loss column travels with [WᵀX | WᵀW] through the exchange, the top combiner of every rank applies
SK:872-884 to the same summed error, and every rank stops at the same iteration.

Two processes share one GPU over gloo (the exchange through IPC-mapped buffers; both grids
co-resident: 64 / 100 workgroups per rank).  Checked: the path taken (exchange + device test on
both ranks), sklearn's n_iter from the fp64 oracle (a stop inside the launch, and a run to
max_iter), identical H on both ranks, W and H at the 1e-5 bar.
"""
import multiprocessing as mp
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


def _data(N, k):
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(N, 81, seed=7, dtype=np.float32)
    W0, H0 = random_init(X, k, 42)
    return X, W0, H0


def _rank_main(rank, world, port, N, k, tol, max_iter, q):
    try:
        import torch
        import torch.distributed as dist
        from cnmf_amd import solver
        from cnmf_amd.distributed import factorise_sharded, shard_bounds
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        seen = []
        orig = solver.MUPlan.prepare_device_tol

        def spy(self, *a, **kw):
            r = orig(self, *a, **kw)
            seen.append((bool(self.exchange), r is not None))
            return r
        solver.MUPlan.prepare_device_tol = spy
        X, W0, H0 = _data(N, k)
        lo, hi = shard_bounds(N, world, rank, align=64)
        W, H, n = factorise_sharded(torch.from_numpy(X[lo:hi]), W0[lo:hi], H0, max_iter=max_iter, tol=tol)
        q.put((rank, W.cpu().numpy(), H.double().cpu().numpy(), n, seen, None))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as ex:  # reported to the parent
        q.put((rank, None, None, None, None, f"{type(ex).__name__}: {ex}"))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("k,N,tol", [(4, 32768, 1e-3), (4, 32768, 1e-4), (8, 25600, 1e-4)],
                         ids=["k4-stop", "k4-max_iter", "k8-stop"])
def test_sharded_fit_with_the_device_tolerance_test(k, N, tol):
    world, max_iter = 2, 400
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, N, k, tol, max_iter, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            r, W, H, n, seen, err = q.get(timeout=400)
            out[r] = (W, H, n, seen, err)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    errs = [v[4] for v in out.values() if v[4]]
    assert not errs, errs
    for r in range(world):
        assert out[r][3] == [(True, True)], out[r][3]  # the exchange AND the device test, one launch
    assert out[0][2] == out[1][2]
    np.testing.assert_array_equal(out[0][1], out[1][1])
    X, W0, H0 = _data(N, k)
    Wr, Hr, nr = mu_ref.mu_fit(X.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                               max_iter=max_iter, tol=tol)
    assert out[0][2] == nr, (out[0][2], nr)
    W = np.concatenate([out[0][0], out[1][0]])
    ew, eh = rel_fro(W, Wr), rel_fro(out[0][1], Hr)
    print(f"k={k} tol={tol}: n_iter {nr}, rel W {ew:.2e} H {eh:.2e}")
    assert ew <= 1e-5 and eh <= 1e-5, (ew, eh)
