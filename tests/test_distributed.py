"""World-size-2 gloo test of the row-sharded MU orchestration on CPU.

The multi-GPU host path (`MUPlan.iterate` / `run_mu` with world > 1: per iteration one shard step
(pending basis update from the all-reduced AB, then the shard's W update and local [WᵀX | WᵀW])
and one all_reduce(AB); a final basis update; the loss check all-reduces one double) runs
unchanged; only the device launches are replaced by a NumPy stand-in (test-only: the product has
no CPU path).  Two ranks on disjoint row shards must reproduce the unsharded oracle fit.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cnmf_amd import _lib
from cnmf_amd.distributed import shard_bounds
from cnmf_amd.solver import MUPlan, WeightedMUPlan, plan_world, run_mu
from oracle import mu_ref, wmu_ref


class _NumpyPlan(MUPlan):
    """MUPlan with the three launches done by the oracle on CPU (fp64)."""

    def __init__(self, X, W, H, group=None, regs=(0.0, 0.0, 0.0, 0.0)):  # noqa: D107 — no super()
        self.X = np.asarray(X, dtype=np.float64)
        self.n_rows, self.F = self.X.shape
        self.k = H.shape[0]
        self.V = self.F + self.k
        self.n_out = self.k * self.V
        self.l1_W, self.l2_W, self.l1_H, self.l2_H = regs
        self.group = group
        self.world = plan_world(group)
        self.shard_steps = False
        self.Wn = np.array(W, dtype=np.float64)
        self.Hn = np.array(H, dtype=np.float64)
        self.AB = torch.zeros(self.n_out, dtype=torch.float64)
        self.loss_buf = torch.zeros(1, dtype=torch.float64)
        self._partial = None

    def sample_pass(self, flags):
        if flags & _lib.PASS_LOSS:
            R = self.X - self.Wn @ self.Hn
            self._partial = np.array([np.sum(R * R)])
            return
        if flags & _lib.PASS_UPDATE_W:
            self.Wn, _, _ = mu_ref.update_w(self.X, self.Wn, self.Hn, self.l1_W, self.l2_W)
        if flags & _lib.PASS_ACCUMULATE:
            A = self.Wn.T @ self.X
            B = self.Wn.T @ self.Wn
            self._partial = np.concatenate([A, B], axis=1).ravel()

    def reduce(self, n_out, out):
        out.copy_(torch.from_numpy(self._partial[:n_out]))

    def shard_step(self, apply_first):  # the contract of cnmf_mu_shard_step
        if apply_first:
            self.basis_update()
        self.sample_pass(_lib.PASS_UPDATE_W | _lib.PASS_ACCUMULATE)
        self.reduce(self.n_out, self.AB)

    def basis_update(self):
        AB = self.AB.numpy().reshape(self.k, self.V)
        self.Hn = mu_ref.update_h_from_accumulators(AB[:, :self.F], AB[:, self.F:], self.Hn,
                                                    self.l1_H, self.l2_H)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, X, W0, H0, max_iter, tol, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = shard_bounds(X.shape[0], world, rank)
        plan = _NumpyPlan(X[lo:hi], W0[lo:hi], H0, group=dist.group.WORLD)
        n_iter = run_mu(plan, max_iter=max_iter, tol=tol)
        out[rank] = (lo, hi, plan.Wn, plan.Hn, n_iter)
    finally:
        dist.destroy_process_group()


def _indep_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cnmf_amd.synthetic import iop_spectra, random_init
        assert plan_world(None) == 1 and plan_world(dist.group.WORLD) == world
        # an independent fit per rank (cNMF replicates under torchrun): different data on each rank,
        # no group passed -> nothing may be all-reduced across the ranks
        X = iop_spectra(200 + 37 * rank, 81, seed=rank, dtype=np.float64)
        W0, H0 = random_init(X, 4, 5 + rank)
        plan = _NumpyPlan(X, W0, H0)
        plan.shard_steps = True  # the shard-step iteration; without a group it all-reduces nothing
        n_iter = run_mu(plan, max_iter=50, tol=1e-3)
        out[rank] = (X, W0, H0, plan.Wn, plan.Hn, n_iter)
    finally:
        dist.destroy_process_group()


def test_plan_without_group_is_a_single_process_fit():
    """a plan built without a group inside an initialised default group fits its
    own rows only (world 1); each rank's result equals the single-process oracle fit of its data."""
    manager = mp.Manager()
    out = manager.dict()
    mp.spawn(_indep_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    for rank in range(2):
        X, W0, H0, W, H, n_iter = out[rank]
        Wr, Hr, nr = mu_ref.mu_fit(X, W0, H0, max_iter=50, tol=1e-3)
        assert n_iter == nr
        np.testing.assert_allclose(H, Hr, rtol=1e-10, atol=1e-14)
        np.testing.assert_allclose(W, Wr, rtol=1e-10, atol=1e-14)


def test_shard_bounds_cover_rows():
    for n, w in [(10, 3), (1_000_000, 8), (7, 8), (0, 2)]:
        b = [shard_bounds(n, w, r) for r in range(w)]
        assert b[0][0] == 0 and b[-1][1] == n
        assert all(b[i][1] == b[i + 1][0] for i in range(w - 1))
        assert max(h - l for l, h in b) - min(h - l for l, h in b) <= 1


@pytest.mark.parametrize("tol,max_iter", [(0.0, 30), (1e-3, 400)])
def test_two_rank_gloo_matches_unsharded(tol, max_iter):
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(301, 81, seed=11, dtype=np.float64)
    W0, H0 = random_init(X, 4, 3)
    manager = mp.Manager()
    out = manager.dict()
    mp.spawn(_worker, args=(2, _free_port(), X, W0, H0, max_iter, tol, out), nprocs=2, join=True)
    Wr, Hr, nr = mu_ref.mu_fit(X, W0, H0, max_iter=max_iter, tol=tol)
    W = np.zeros_like(W0)
    for rank in range(2):
        lo, hi, Wp, Hp, n_iter = out[rank]
        W[lo:hi] = Wp
        assert n_iter == nr
        np.testing.assert_allclose(Hp, Hr, rtol=1e-10, atol=1e-14)
    np.testing.assert_allclose(W, Wr, rtol=1e-10, atol=1e-14)


class _NumpyWeightedPlan(WeightedMUPlan):
    """WeightedMUPlan with its launches done by the weighted oracle on CPU (fp64)."""

    def __init__(self, X, M, W, H, group=None):  # noqa: D107 — no super(): no HIP buffers
        self.X = np.asarray(X, dtype=np.float64)
        self.Mw = np.asarray(M, dtype=np.float64)
        self.n_rows, self.F = self.X.shape
        self.k = H.shape[0]
        self.n_out = 2 * self.k * self.F
        self.group = group
        self.world = plan_world(group)
        self.Wn = np.array(W, dtype=np.float64)
        self.Hn = np.array(H, dtype=np.float64)
        self.AD = torch.zeros(self.n_out, dtype=torch.float64)
        self.loss_buf = torch.zeros(1, dtype=torch.float64)
        self._partial = None

    def sample_pass(self, flags):
        if flags & _lib.PASS_LOSS:
            R = self.X - self.Wn @ self.Hn
            self._partial = np.array([np.sum(self.Mw * R * R)])
            return
        self.Wn = wmu_ref.update_w(self.X, self.Mw, self.Wn, self.Hn)
        if flags & _lib.PASS_ACCUMULATE:
            A = self.Wn.T @ (self.Mw * self.X)
            D = self.Wn.T @ (self.Mw * (self.Wn @ self.Hn))
            self._partial = np.concatenate([A.ravel(), D.ravel()])

    def reduce(self, n_out, out):
        out.copy_(torch.from_numpy(self._partial[:n_out]))

    def basis_update(self):
        AD = self.AD.numpy()
        kF = self.k * self.F
        A, D = AD[:kF].reshape(self.k, self.F), AD[kF:].reshape(self.k, self.F).copy()
        D[D == 0] = wmu_ref.EPSILON
        self.Hn = self.Hn * (A / D)


def _wworker(rank, world, port, X, M, W0, H0, max_iter, tol, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = shard_bounds(X.shape[0], world, rank)
        plan = _NumpyWeightedPlan(X[lo:hi], M[lo:hi], W0[lo:hi], H0, group=dist.group.WORLD)
        n_iter = run_mu(plan, max_iter=max_iter, tol=tol)
        out[rank] = (lo, hi, plan.Wn, plan.Hn, n_iter)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("tol,max_iter", [(0.0, 30), (1e-3, 400)])
def test_two_rank_gloo_weighted_matches_unsharded(tol, max_iter):
    """The weighted MU's host path (WeightedMUPlan.iterate + run_mu at world 2: one all_reduce of the
    2kF accumulators per iteration, one double per error check) reproduces the unsharded oracle."""
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(301, 81, seed=12, dtype=np.float64)
    rng = np.random.default_rng(5)
    M = rng.uniform(0.2, 2.0, X.shape) * (rng.random(X.shape) >= 0.3)
    W0, H0 = random_init(X, 4, 3)
    manager = mp.Manager()
    out = manager.dict()
    mp.spawn(_wworker, args=(2, _free_port(), X, M, W0, H0, max_iter, tol, out), nprocs=2, join=True)
    Wr, Hr, nr = wmu_ref.wmu_fit(X, M, W0, H0, max_iter=max_iter, tol=tol)
    W = np.zeros_like(W0)
    for rank in range(2):
        lo, hi, Wp, Hp, n_iter = out[rank]
        W[lo:hi] = Wp
        assert n_iter == nr
        np.testing.assert_allclose(Hp, Hr, rtol=1e-10, atol=1e-14)
    np.testing.assert_allclose(W, Wr, rtol=1e-10, atol=1e-14)


class _FlakyExchangePlan(_NumpyPlan):
    """A multi-GPU plan on the persistent in-launch-exchange path whose FIRST launch fails on rank 0
    only: its error word is set and its results are invalid (W scaled), while rank 1's
    launch completed with valid results.  The in-launch exchange is modelled by one all_reduce per
    iteration, so the collectives of both ranks stay paired however the fallback goes."""

    def __init__(self, *a, rank=0, **kw):
        super().__init__(*a, **kw)
        self.rank = rank
        self.persistent = self.persistent_shape = self.exchange = True
        self.device = torch.device("cpu")
        self._fail_next = rank == 0
        self._err = False
        self.W = torch.zeros(1)  # snapshot targets of _iterate_guarded (mirrors Wn / Hn below)
        self.H64 = torch.zeros(1)
        self.fallbacks = 0

    def iterate(self, n_iter, update_H=True, pass_events=None):
        if not self.exchange:
            self.fallbacks += 1
        for i in range(n_iter):
            self.shard_step(apply_first=i > 0)
            self._allreduce(self.AB)
        self.basis_update()
        if self.exchange and self._fail_next:
            self._fail_next, self._err = False, True
            self.Wn = self.Wn * 2.0  # the failed launch's results are invalid

    def prepare_device_tol(self, *a, **kw):
        return None  # the host-checked stretches (the path this test exercises)

    def check_sync_error(self):
        if self._err:
            self._err = False
            self.disable_exchange()
            raise _lib.HipLibraryError("multi-GPU persistent launch failed (forced on one rank)")

    def _allreduce(self, t):
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.SUM, group=self.group)

    def disable_exchange(self):
        self.exchange = False

    def refresh_basis(self):
        pass


def _snapshotting(plan):
    """Route _iterate_guarded's W / H64 snapshot and restore through the NumPy state."""
    class _T:
        def __init__(self, get, put):
            self.get, self.put = get, put

        def clone(self):
            return self.get().copy()

        def copy_(self, v):
            self.put(v.copy())
    plan.W = _T(lambda: plan.Wn, lambda v: setattr(plan, "Wn", v))
    plan.H64 = _T(lambda: plan.Hn, lambda v: setattr(plan, "Hn", v))
    return plan


def _flaky_worker(rank, world, port, X, W0, H0, out):
    import warnings
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = shard_bounds(X.shape[0], world, rank)
        plan = _snapshotting(_FlakyExchangePlan(X[lo:hi], W0[lo:hi], H0, group=dist.group.WORLD, rank=rank))
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            n_iter = run_mu(plan, max_iter=30, tol=1e-3)
        out[rank] = (lo, hi, plan.Wn, plan.Hn, n_iter, plan.fallbacks, plan.exchange)
    finally:
        dist.destroy_process_group()


def test_failed_launch_on_one_rank_falls_back_on_every_rank():
    """a persistent multi-GPU launch that fails on ONE rank makes EVERY rank
    restore its snapshot and re-run the stretch on the RCCL path (a collective verdict): both ranks
    end on the unsharded oracle's factors with identical H and the same n_iter."""
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(257, 81, seed=21, dtype=np.float64)
    W0, H0 = random_init(X, 4, 9)
    manager = mp.Manager()
    out = manager.dict()
    mp.spawn(_flaky_worker, args=(2, _free_port(), X, W0, H0, out), nprocs=2, join=True)
    Wr, Hr, nr = mu_ref.mu_fit(X, W0, H0, max_iter=30, tol=1e-3)
    W = np.zeros_like(W0)
    for rank in range(2):
        lo, hi, Wp, Hp, n_iter, fallbacks, exchange = out[rank]
        W[lo:hi] = Wp
        assert n_iter == nr and fallbacks >= 1 and not exchange
        np.testing.assert_allclose(Hp, Hr, rtol=1e-10, atol=1e-14)
    np.testing.assert_array_equal(out[0][3], out[1][3])
    np.testing.assert_allclose(W, Wr, rtol=1e-10, atol=1e-14)
