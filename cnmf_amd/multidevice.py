"""Several GPUs driven from ONE process: `factorise(X, ..., devices=[...])`.

The rows of X are split into one contiguous shard per entry of `devices` (64-row aligned, as the
multi-process path shards them: cnmf_amd.distributed.shard_bounds).  Each shard gets its own plan
on its device and its own host thread and stream; the threads run the same driver (`run_mu`), and
the plans' collectives go through a `LocalGroup` instead of torch.distributed:

* the in-launch exchange (persistent shapes): every stretch of iterations is ONE persistent launch
  per shard whose [WᵀX | WᵀW] all-reduce happens inside the launches, over exchange buffers mapped
  directly into every device (peer access; no IPC inside one process) — the multi-process
  exchange's protocol and kernels (cnmf_mu_iterations_multi);
* otherwise (other shapes, or shards sharing a device whose persistent grids would not all be
  resident together): one shard step per iteration and a host-side all-reduce of the small
  accumulators (summed in shard order: the same bits on every shard).

The host thread per device only issues launches; the GIL is released while a thread waits on its
device.  Results equal the one-device fit to fp64 summation order (tests/test_gpu_multidevice.py).
Entries of `devices` may repeat (two logical shards on one GPU, e.g. for testing): those shards
take the host all-reduce path by default, because HIP does not promise that two launches on
different streams of ONE device run concurrently (streams share the device's few hardware queues),
and the exchange needs every shard's launch resident at once; `shared_device_exchange=True` tries
it anyway when the grids fit together (a launch that waits in vain times out and every shard
falls back to the host all-reduce, with the same result).
"""
from __future__ import annotations

import threading
import warnings

import numpy as np
import torch

from . import _lib
from .distributed import shard_bounds

__all__ = ["LocalGroup", "factorise_devices"]


class LocalGroup:
    """The collectives a plan uses (sum / max all-reduce of a small tensor, all-gather of objects)
    among the P shards of one process, each driven by its own thread.  `view(rank)` is the handle a
    plan holds (`plan.group`): it knows its rank.  Every collective is a rendezvous of all P
    threads; a thread that fails aborts the barrier so that the others raise instead of waiting."""

    is_local = True

    def __init__(self, size: int):
        self._size = int(size)
        self._barrier = threading.Barrier(self._size)
        self._slots = [None] * self._size

    def view(self, rank: int) -> "_LocalView":
        return _LocalView(self, rank)

    def abort(self):
        self._barrier.abort()

    def reset(self):
        """Make the group usable again after an abort (call once every thread has left it)."""
        self._barrier.reset()
        self._slots = [None] * self._size

    def _exchange(self, rank: int, obj):
        self._slots[rank] = obj
        self._barrier.wait()
        out = list(self._slots)
        self._barrier.wait()  # every thread has read the slots before they are reused
        return out


class _LocalView:
    is_local = True

    def __init__(self, group: LocalGroup, rank: int):
        self._g, self._rank = group, rank

    def size(self) -> int:
        return self._g._size

    def rank(self) -> int:
        return self._rank

    def all_gather(self, obj) -> list:
        return self._g._exchange(self._rank, obj)

    def all_reduce(self, t: torch.Tensor, op: str = "sum"):
        """In place; the shards' values combined in shard order in fp64 on the host (identical bits
        on every shard)."""
        parts = self._g._exchange(self._rank, t.detach().to("cpu", torch.float64).clone())
        acc = parts[0].clone()
        for p in parts[1:]:
            acc = acc + p if op == "sum" else torch.maximum(acc, p)
        t.copy_(acc.to(t.dtype))

    def all_reduce_values(self, values, op: str = "max") -> list:
        t = torch.tensor([float(v) for v in values], dtype=torch.float64)
        self.all_reduce(t, op)
        return [float(v) for v in t.tolist()]


def _device(d) -> torch.device:
    if isinstance(d, torch.device):
        return d if d.index is not None else torch.device("cuda", torch.cuda.current_device())
    if isinstance(d, str):
        return _device(torch.device(d))
    return torch.device("cuda", int(d))


def _exchange_fits(plans, shared_device_exchange=False) -> bool:
    """Every shard a persistent shape, and on each device the shards' persistent grids together
    within the CUs (one resident wave-tile workgroup per CU): co-running launches on one device all
    have to be resident, or the exchange would wait for a launch that cannot start."""
    if not all(getattr(p, "exchange_shape", False) for p in plans):
        return False
    if len({p.device.index for p in plans}) < len(plans) and not shared_device_exchange:
        return False
    if not all(type(p).__name__ == "MUPlan" for p in plans):
        return len({p.device.index for p in plans}) == len(plans)  # ALS / weighted: distinct devices
    per_dev = {}
    for p in plans:
        with torch.cuda.device(p.device):
            g = int(p.lib.cnmf_persist_workgroups(p.n_rows, p.F, p.k, p.xdt, p.layout, 1))
        if g <= 0:
            return False
        per_dev[p.device.index] = per_dev.get(p.device.index, 0) + g
    return all(n <= torch.cuda.get_device_properties(d).multi_processor_count for d, n in per_dev.items())


class MultiDeviceFit:
    """The shard plans of one fit over `devices` and the threads that drive them."""

    def __init__(self, X, Mw, k, regs, devices, *, solver="mu", sum_to_one=None, smoothness=0.0,
                 align=64, shared_device_exchange=False):
        from .api import _make_plan
        self.devices = [_device(d) for d in devices]
        P = len(self.devices)
        if P < 1:
            raise ValueError("devices must name at least one HIP device")
        n = int(X.shape[0])
        self.group = LocalGroup(P)
        self.bounds = [shard_bounds(n, P, r, align=align) for r in range(P)]
        self.plans = []
        for r, (dev, (lo, hi)) in enumerate(zip(self.devices, self.bounds)):
            with torch.cuda.device(dev):
                self.plans.append(_make_plan(X[lo:hi], None if Mw is None else Mw[lo:hi], k, regs, dev,
                                             solver=solver, sum_to_one=sum_to_one, smoothness=smoothness,
                                             group=self.group.view(r)))
        self.streams = [torch.cuda.Stream(p.device) for p in self.plans]
        self.exchange = False
        self.shared_device_exchange = bool(shared_device_exchange)

    def _run(self, fn):
        """fn(rank, plan) on every shard's thread, with its device and stream current; re-raises the
        first failure (after the other threads have been released from any rendezvous)."""
        errs = [None] * len(self.plans)

        def body(r):
            try:
                torch.cuda.set_device(self.plans[r].device)
                with torch.cuda.stream(self.streams[r]):
                    fn(r, self.plans[r])
                    torch.cuda.current_stream().synchronize()
            except BaseException as e:  # noqa: BLE001 — reported below
                errs[r] = e
                self.group.abort()

        threads = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(len(self.plans))]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        if any(errs):  # every thread has left the rendezvous: the group serves the fallback path
            self.group.reset()
        first = [e for e in errs if e is not None and not isinstance(e, threading.BrokenBarrierError)]
        if first or any(errs):
            raise first[0] if first else errs[0]

    def start(self, W, H, avg):
        from .api import _start

        def go(r, plan):
            lo, hi = self.bounds[r]
            _start(plan, None if W is None else W[lo:hi], H, avg)
        self._run(go)

    def enable_exchange(self):
        if len(self.plans) == 1 or not _exchange_fits(self.plans, self.shared_device_exchange):
            return False
        try:
            self._run(lambda r, plan: plan.enable_exchange())
        except _lib.HipLibraryError as e:
            warnings.warn(f"in-launch exchange not used: {e}", RuntimeWarning)
            return False
        self.exchange = all(p.exchange for p in self.plans)
        return self.exchange

    def run(self, max_iter, tol, update_H=True, verbose=0):
        from .solver import run_mu
        n = [None] * len(self.plans)

        def go(r, plan):
            n[r] = run_mu(plan, max_iter=max_iter, tol=tol, update_H=update_H, verbose=verbose if r == 0 else 0)
        self._run(go)
        assert len(set(n)) == 1, n
        return n[0]

    def normalise(self, norm):
        self._run(lambda r, plan: plan.normalise(norm))

    def release(self):
        self._run(lambda r, plan: torch.cuda.synchronize(plan.device))
        for p in self.plans:
            rel = getattr(p, "release", None)
            if rel is not None:
                rel()

    def W(self, device=None) -> torch.Tensor:
        dev = device or self.plans[0].device
        return torch.cat([p.W.to(dev) for p in self.plans], dim=0)

    def H(self) -> torch.Tensor:
        return self.plans[0].H()


def factorise_devices(X, W, H, n_components, *, devices, init=None, update_H=True, solver="mu",
                      tol=1e-4, max_iter=200, alpha_W=0.0, alpha_H="same", l1_ratio=0.0,
                      random_state=None, verbose=0, normalise=None, sum_to_one=None, smoothness=0.0,
                      weights=None, init_device="auto"):
    """`factorise(..., devices=[...])`: the fit of `cnmf_amd.api.factorise` with the rows split over
    the listed devices of this process.  Returns (W, H, n_iter) like factorise (NumPy in, NumPy out;
    torch in: tensors on devices[0])."""
    from .api import ConvergenceWarning, _out, _resolve, _transform_start
    devs = [_device(d) for d in devices]
    X, Mw, as_torch, streamed, k, W, H, regs = _resolve(
        X, W, H, n_components, init, update_H, alpha_W, alpha_H, l1_ratio, random_state, devs[0],
        solver=solver, normalise=normalise, weights=weights, init_device=init_device)
    fit = MultiDeviceFit(X, Mw, k, regs, devs, solver=solver, sum_to_one=sum_to_one, smoothness=smoothness)
    try:
        fit.start(W, H, _transform_start(X, as_torch, k) if W is None else None)
        if update_H:
            fit.enable_exchange()
        n_iter = fit.run(max_iter, tol, update_H=update_H, verbose=verbose)
        if n_iter == max_iter and tol > 0:
            warnings.warn("Maximum number of iterations %d reached. Increase it to improve "
                          "convergence." % max_iter, ConvergenceWarning)
        if normalise is not None and update_H:
            fit.normalise(normalise)
        Wd, Hd = fit.W(), fit.H()
        return _out(Wd, as_torch, X), _out(Hd, as_torch, X), n_iter
    finally:
        fit.release()
