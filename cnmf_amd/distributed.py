"""Row-sharded MU across GPUs: one process per GPU, torch.distributed over RCCL.

Each rank owns a contiguous block of rows of X and W; H is replicated.  Per iteration every rank runs
the fused pass on its shard, reduces its per-workgroup partials to the k·(F+k) fp64 accumulators
[WᵀX | WᵀW], ONE all_reduce(SUM) combines them over xGMI (backend "nccl" is RCCL on ROCm), and every
rank applies the identical fp64 basis update — no broadcast.  The error check every 10 iterations
all-reduces one double.  The sharding is exact: Σ_p W_pᵀX_p = WᵀX (tests/test_distributed.py).

    import torch.distributed as dist
    dist.init_process_group("nccl")
    lo, hi = shard_bounds(n_rows, dist.get_world_size(), dist.get_rank())
    W_r, H, n_iter = factorise_sharded(X[lo:hi], W0[lo:hi], H0, max_iter=500, tol=0)
"""
from __future__ import annotations

import warnings

import torch
import torch.distributed as dist

from . import _lib
from .solver import ALSPlan, MUPlan, WeightedMUPlan, run_mu

__all__ = ["shard_bounds", "factorise_sharded"]


def shard_bounds(n_rows: int, world: int, rank: int, align: int = 1):
    """Contiguous, balanced [lo, hi) row range of `rank`.  Rows are dealt in blocks of `align` rows
    (the first blocks % world ranks get one block more; the last rank also takes the n_rows % align
    remainder), so with align=64 every shard but possibly the last is a whole number of the
    persistent kernels' 64-row tiles."""
    n_rows, world, align = int(n_rows), int(world), max(1, int(align))
    nb = n_rows // align
    base, extra = divmod(nb, world)
    lo = (rank * base + min(rank, extra)) * align
    hi = lo + (base + (1 if rank < extra else 0)) * align
    if rank == world - 1:
        hi = n_rows
    return lo, hi


def factorise_sharded(X_shard, W_shard, H0, *, max_iter=200, tol=1e-4, l1_reg_W=0.0, l2_reg_W=0.0,
                      l1_reg_H=0.0, l2_reg_H=0.0, update_H=True, group=None, device=None,
                      exchange="auto", weights=None, solver="mu", sum_to_one=0.0, smoothness=0.0):
    """MU on this rank's rows; returns (W_shard, H, n_iter) as device tensors.

    X_shard: (n_r, F) float32/float64/bfloat16 tensor (any device; moved to `device`, default the
    current HIP device), W_shard: (n_r, k), H0: (k, F) identical on every rank (broadcast from rank 0
    here to make that true).  Regularisation constants are the already-scaled sklearn l1/l2 terms
    (SK:1254-1265 computed on the GLOBAL n_samples).

    exchange='auto' (default): run each stretch of iterations as ONE persistent launch per rank with
    the all-reduce inside the launch (peer exchange over xGMI, MUPlan.enable_exchange) when every
    shard is a persistent shape — fp32, F = 81, MU k = 4 or 8 (shard rows a multiple of 16 / 8),
    the constrained ALS and the weighted MU at k = 4 (rows a multiple of 16) — and the buffers can
    be shared; otherwise the RCCL path (one shard step + one all_reduce per iteration).
    exchange=True: the same, with a warning when it falls back; exchange=False: always RCCL.
    A launch that fails on any rank sends every rank back to the RCCL path (solver.sync_failed).

    weights: this rank's rows of the per-element weights (float32 X): the
    weighted / masked MU, whose 2kF accumulators [W'ᵀ(M∘X) | W'ᵀ(M∘(W'H))] are all-reduced the
    same way (no regularisation).
    solver='als': the constrained ALS (sum_to_one, smoothness), its [WᵀX | WᵀW]
    all-reduced before every H-step.  Both take exchange=True (fp32, F = 81, k = 4, rows a multiple
    of 16): one persistent launch per rank with the all-reduce inside it.
    """
    if exchange not in ("auto", True, False):
        raise ValueError(f"exchange must be 'auto', True or False, got {exchange!r}")
    if not (dist.is_available() and dist.is_initialized()):
        raise RuntimeError("factorise_sharded needs an initialised torch.distributed process group")
    group = group if group is not None else dist.group.WORLD
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    X = torch.as_tensor(X_shard).to(dev).contiguous()
    H0 = torch.as_tensor(H0).to(dev, torch.float64).contiguous()
    dist.broadcast(H0, src=dist.get_global_rank(group, 0), group=group)
    if solver not in ("mu", "als"):
        raise ValueError(f"solver must be 'mu' or 'als', got {solver!r}")
    if weights is not None or solver == "als":
        if any((l1_reg_W, l2_reg_W, l1_reg_H, l2_reg_H)):
            raise ValueError("the weighted MU and the constrained ALS take no l1/l2 regularisation")
        if weights is not None and solver == "als":
            raise ValueError("weights apply to solver='mu'")
    if weights is not None:
        M = torch.as_tensor(weights).to(dev, torch.float32).contiguous()
        plan = WeightedMUPlan(X, M, H0.shape[0], group=group)
    elif solver == "als":
        plan = ALSPlan(X, H0.shape[0], sum_to_one=sum_to_one, smoothness=smoothness, group=group)
    else:
        plan = MUPlan(X, H0.shape[0], l1_reg_W, l2_reg_W, l1_reg_H, l2_reg_H, group=group)
    plan.set_W(torch.as_tensor(W_shard))
    plan.set_H(H0)
    if exchange == "auto" and update_H:
        # every rank must take the same decision before the collective enable_exchange
        from .solver import agree_max
        if agree_max([0.0 if plan.exchange_shape else 1.0], group, plan.device)[0] != 0.0:
            exchange = False
    if exchange and update_H:
        try:
            plan.enable_exchange()
        except _lib.HipLibraryError as e:
            if exchange is True:
                warnings.warn(f"in-launch exchange not used: {e}", RuntimeWarning)
    n_iter = run_mu(plan, max_iter=max_iter, tol=tol, update_H=update_H)
    plan.release()
    return plan.W, plan.H(), n_iter
