"""The caller-facing boundary: sklearn-shaped `factorise` / `fit` / `non_negative_factorization`
and the `NMF` estimator, with the argument meaning, defaults and error behaviour of
scikit-learn 1.7.2's Frobenius MU path (SK = sklearn/decomposition/_nmf.py):

  non_negative_factorization   SK:905-1131   -> factorise (aliases fit, non_negative_factorization)
  NMF.fit_transform/transform  SK:1600-1763  -> NMF
  _check_init / _check_w_h      SK:68-82, SK:1194-1252
  _compute_regularization       SK:1254-1265
  _initialize_nmf ('random')    SK:303-314   (nndsvd / nndsvda / nndsvdar: cnmf_amd.init)

Differences, all deliberate: the solvers are 'mu' (the default here; sklearn's default 'cd'
raises) and the build's constrained ALS 'als' (sum_to_one / smoothness; k ≤ 4),
only beta_loss='frobenius' is accepted, sparse X is not, and n_components ≤ 16.  normalise=
('l1' | 'l2' | 'max') adds the §8 a6 projection (off by default, so 'mu' output is sklearn's).  NumPy
inputs are copied to the GPU and results come back as NumPy arrays of X's dtype; torch tensors on a
HIP device stay there (fp32, fp64 or bf16 X; bf16 computes in fp32 and returns fp32 W/H).
There is no CPU fallback: without the HIP library every call raises HipLibraryError.
"""
from __future__ import annotations

import numbers
import warnings

import numpy as np

from . import init as _init
from .synthetic import random_init

__all__ = ["factorise", "fit", "non_negative_factorization", "NMF", "ConvergenceWarning"]

class ConvergenceWarning(UserWarning):
    """Custom warning to capture convergence problems (the role of
    sklearn.exceptions.ConvergenceWarning; the product path imports nothing from sklearn)."""

_INITS = {"random", "nndsvd", "nndsvda", "nndsvdar", "custom", None}


def _torch():
    import torch
    return torch


def _is_torch(a) -> bool:
    try:
        import torch
    except Exception:  # pragma: no cover
        return False
    return isinstance(a, torch.Tensor)


# ------------------------------------------------------------------------------------------------
# validation (messages follow sklearn's)
# ------------------------------------------------------------------------------------------------
def _check_X(X):
    if _is_torch(X):
        torch = _torch()
        if X.dim() != 2:
            raise ValueError(f"Expected 2D array, got {X.dim()}D array instead")
        if X.dtype not in (torch.float32, torch.float64, torch.bfloat16):
            X = X.to(torch.float64)
        if not bool(torch.isfinite(X).all()):
            raise ValueError("Input X contains NaN or infinity.")
        return X if X.device.type != "cpu" else X.contiguous()  # host rows are streamed / copied row-major
    X = np.asarray(X)
    if X.ndim != 2:
        raise ValueError(f"Expected 2D array, got {X.ndim}D array instead")
    if X.dtype not in (np.float32, np.float64):
        X = X.astype(np.float64)
    if X.shape[0] < 1 or X.shape[1] < 1:
        raise ValueError(f"Found array with shape {X.shape}; a minimum of 1 is required.")
    step = max(1, (1 << 26) // X.shape[1])  # row blocks: a memory-mapped X is never held whole
    for lo in range(0, X.shape[0], step):
        if not np.isfinite(X[lo:lo + step]).all():
            raise ValueError("Input X contains NaN or infinity.")
    return np.ascontiguousarray(X)


def _min(a):
    return float(a.min()) if not _is_torch(a) else float(a.min().item())


def _max(a):
    return float(a.max()) if not _is_torch(a) else float(a.max().item())


def _check_non_negative(A, whom):
    if _min(A) < 0:
        raise ValueError(f"Negative values in data passed to {whom}.")


def _check_init(A, shape, whom):
    """SK:68-82."""
    if A is None:
        raise ValueError(f"{whom} must be provided when init='custom'")
    A = A if _is_torch(A) else np.asarray(A)
    if A.ndim != 2:
        raise ValueError(f"Expected 2D array, got {A.ndim}D array instead")
    if shape[0] != "auto" and A.shape[0] != shape[0]:
        raise ValueError(f"Array with wrong first dimension passed to {whom}. Expected {shape[0]}, "
                         f"but got {A.shape[0]}.")
    if shape[1] != "auto" and A.shape[1] != shape[1]:
        raise ValueError(f"Array with wrong second dimension passed to {whom}. Expected {shape[1]}, "
                         f"but got {A.shape[1]}.")
    _check_non_negative(A, whom)
    if _max(A) == 0:
        raise ValueError(f"Array passed to {whom} is full of zeros.")
    return A


def _dtype_name(a):
    return str(a.dtype).replace("torch.", "")


def _validate_params(n_components, init, solver, beta_loss, tol, max_iter, alpha_W, alpha_H,
                     l1_ratio):
    if not (n_components is None or n_components == "auto" or
            (isinstance(n_components, numbers.Integral) and not isinstance(n_components, bool)
             and n_components >= 1)):
        raise ValueError(f"The 'n_components' parameter must be an int in the range [1, inf), "
                         f"None or 'auto'. Got {n_components!r} instead.")
    if init not in _INITS:
        raise ValueError(f"The 'init' parameter must be a str among {{'custom', 'nndsvd', "
                         f"'nndsvda', 'nndsvdar', 'random'}} or None. Got {init!r} instead.")
    if solver not in ("mu", "als"):
        raise ValueError(f"solver={solver!r} is not available: this build implements the "
                         "multiplicative-update solver ('mu') and the constrained ALS ('als').")
    if beta_loss not in ("frobenius", 2, 2.0):
        raise ValueError(f"beta_loss={beta_loss!r} is not available: only 'frobenius' (2) is "
                         "implemented on the MI355X path.")
    if not isinstance(tol, numbers.Real) or tol < 0:
        raise ValueError(f"The 'tol' parameter must be a float in the range [0, inf). Got {tol!r} instead.")
    if not isinstance(max_iter, numbers.Integral) or isinstance(max_iter, bool) or max_iter < 1:
        raise ValueError(f"The 'max_iter' parameter must be an int in the range [1, inf). "
                         f"Got {max_iter!r} instead.")
    if not isinstance(alpha_W, numbers.Real) or alpha_W < 0:
        raise ValueError(f"The 'alpha_W' parameter must be a float in the range [0, inf). Got {alpha_W!r} instead.")
    if not (alpha_H == "same" or (isinstance(alpha_H, numbers.Real) and alpha_H >= 0)):
        raise ValueError(f"The 'alpha_H' parameter must be a float in the range [0, inf) or a str "
                         f"among {{'same'}}. Got {alpha_H!r} instead.")
    if not isinstance(l1_ratio, numbers.Real) or not 0 <= l1_ratio <= 1:
        raise ValueError(f"The 'l1_ratio' parameter must be a float in the range [0, 1]. Got {l1_ratio!r} instead.")


def _compute_regularization(n_samples, n_features, alpha_W, alpha_H, l1_ratio):
    """SK:1254-1265."""
    alpha_H = alpha_W if alpha_H == "same" else alpha_H
    return (n_features * alpha_W * l1_ratio, n_samples * alpha_H * l1_ratio,
            n_features * alpha_W * (1.0 - l1_ratio), n_samples * alpha_H * (1.0 - l1_ratio))


# ------------------------------------------------------------------------------------------------
# the core fit
# ------------------------------------------------------------------------------------------------
def _validate_als(solver, alpha_W, alpha_H, sum_to_one, smoothness):
    if solver != "als":
        if sum_to_one is not None or smoothness:
            raise ValueError("sum_to_one / smoothness apply to solver='als' only")
        return
    if alpha_W != 0 or alpha_H not in ("same", 0, 0.0):
        raise ValueError("solver='als' takes no alpha_W / alpha_H regularisation (use sum_to_one "
                         "and smoothness)")
    for name, v in (("sum_to_one", sum_to_one), ("smoothness", smoothness)):
        if v is not None and (not isinstance(v, numbers.Real) or v < 0):
            raise ValueError(f"The '{name}' parameter must be a float in the range [0, inf) or None. "
                             f"Got {v!r} instead.")


def _validate_weights(weights, X, solver, alpha_W, alpha_H, normalise):
    """Weighted / masked MU: per-element weights of X's shape, finite and
    non-negative, float32 X; solver 'mu' without alpha regularisation or normalise."""
    if weights is None:
        return None
    if solver != "mu":
        raise ValueError("weights apply to solver='mu' only")
    if alpha_W != 0 or alpha_H not in ("same", 0, 0.0):
        raise ValueError("the weighted MU takes no alpha_W / alpha_H regularisation")
    if normalise is not None:
        raise ValueError("normalise is not supported together with weights")
    Mw = _check_X(weights)
    if tuple(Mw.shape) != tuple(X.shape):
        raise ValueError(f"weights must have X's shape {tuple(X.shape)}, got {tuple(Mw.shape)}")
    if _min(Mw) < 0:
        raise ValueError("Negative values in data passed to NMF (input weights)")
    torch = _torch()
    if (_is_torch(X) and X.dtype != torch.float32) or (not _is_torch(X) and X.dtype != np.float32):
        raise TypeError("the weighted MU runs in float32: pass X (and W, H) as float32")
    return Mw


_TORCH_DT = {}  # numpy scalar type -> torch dtype, filled on first use
GPU_INIT_MIN_ROWS = 65536


def _streamed(X, as_torch, memory_budget, solver, Mw):
    """Out-of-core when a host X is larger than `memory_budget` bytes."""
    if memory_budget is None:
        return False
    if not isinstance(memory_budget, numbers.Integral) or memory_budget <= 0:
        raise ValueError(f"memory_budget must be a positive number of bytes, got {memory_budget!r}")
    if as_torch and X.device.type != "cpu":
        return False  # already in HBM
    nbytes = X.numel() * X.element_size() if as_torch else X.nbytes
    if nbytes <= memory_budget:
        return False
    if solver != "mu" or Mw is not None:
        raise ValueError("memory_budget (out-of-core streaming) serves the unweighted 'mu' solver")
    if as_torch and X.dtype not in (_torch().float32, _torch().float64):
        raise TypeError("out-of-core streaming takes float32 / float64 X")
    return True  # below this the host init costs less than a device round trip


def _validate_init_device(init_device):
    if init_device not in ("auto", "host", "gpu"):
        raise ValueError(f"The 'init_device' parameter must be a str among {{'auto', 'host', 'gpu'}}. "
                         f"Got {init_device!r} instead.")


def _initial_factors(X, k, init, random_state, device, as_torch, group, host_only=False,
                     init_device="auto"):
    """_initialize_nmf (SK:221-373).

    init_device='host': the host restatement (cnmf_amd.init), bit-identical to sklearn's
    _initialize_nmf on the same BLAS (pinned by tests/golden/init_*.npz).
    init_device='gpu': the NNDSVD family's passes over X on the GPU (cnmf_amd.gpu_init, §8 f4) for a
    tall X of one process (>= GPU_INIT_MIN_ROWS rows, F <= 96, k <= 16); its range finder works in
    fp64 on the Gram matrix, so for float32 X it does NOT reproduce sklearn's float32 randomized SVD:
    on ill-conditioned trailing directions the starts differ at the 1e-3 level (measured: 1.4e-3
    relative on W at 1e6 synthetic rows, tests/test_gpu_init.py), and so do the fitted factors.
    init_device='auto' (default): the GPU init for float64 X (where it agrees with sklearn's fp64
    answer to ~1e-8), the host restatement for float32 / bfloat16 X, so that the default fit
    reproduces the reference's factors.  'random', small X, sharded fits (X is one shard of the
    global matrix) and out-of-core fits always take the host restatement."""
    torch = _torch()
    from . import gpu_init as _gpu_init
    if not _TORCH_DT:
        _TORCH_DT.update({np.float32: torch.float32, np.float64: torch.float64})
    n_samples, n_features = X.shape
    resolved = init
    if init is None:
        resolved = "nndsvda" if k <= min(n_samples, n_features) else "random"
    xdt = X.dtype if as_torch else _TORCH_DT.get(X.dtype.type)
    want_gpu = init_device == "gpu" or (init_device == "auto" and xdt == torch.float64)
    if (want_gpu and group is None and not host_only and n_samples >= GPU_INIT_MIN_ROWS
            and X.min() >= 0 and _gpu_init.gpu_init_eligible(n_samples, n_features, k, resolved, xdt)):
        dev = torch.device(device) if device is not None else (
            X.device if as_torch and X.device.type == "cuda" else torch.device("cuda", torch.cuda.current_device()))
        Xd = (X if as_torch else torch.from_numpy(X)).to(dev).contiguous()
        return _gpu_init.initialize_nmf_gpu(Xd, k, init=resolved, random_state=random_state)
    Xh = X if not as_torch else X.detach().to("cpu", torch.float32 if X.dtype == torch.bfloat16 else X.dtype).numpy()
    return _init.initialize_nmf(Xh, k, init=init, random_state=random_state)


def _resolve(X, W, H, n_components, init, update_H, alpha_W, alpha_H, l1_ratio, random_state, device,
             group=None, solver="mu", normalise=None, weights=None, memory_budget=None,
             init_device="auto"):
    """Validation, k, the starting factors and the regularisation of `_BaseNMF._fit_transform`
    (SK:1638-1712, _check_w_h SK:1194-1252, _compute_regularization SK:1254-1265).  Returns
    (X, Mw, as_torch, streamed, k, W, H, regs); W is None for the update_H=False start."""
    torch = _torch()
    X = _check_X(X)
    Mw = _validate_weights(weights, X, solver, alpha_W, alpha_H, normalise)
    as_torch = _is_torch(X)
    streamed = _streamed(X, as_torch, memory_budget, solver, Mw)
    n_samples, n_features = X.shape
    k = n_components
    if k is None:
        k = n_features
    if k == "auto":
        if init == "custom" or not update_H:
            k = "auto"
        else:
            k = n_features

    # _check_w_h (SK:1194-1252)
    if init == "custom" and update_H:
        H = _check_init(H, (k, n_features), "NMF (input H)")
        W = _check_init(W, (n_samples, k), "NMF (input W)")
        if k == "auto":
            k = H.shape[0]
        if H.dtype != X.dtype or W.dtype != X.dtype:
            if not (as_torch and X.dtype == torch.bfloat16):
                raise TypeError("H and W should have the same dtype as X. Got H.dtype = {} and "
                                "W.dtype = {}.".format(_dtype_name(H), _dtype_name(W)))
    elif not update_H:
        if W is not None:
            warnings.warn("When update_H=False, the provided initial W is not used.", RuntimeWarning)
        H = _check_init(H, (k, n_features), "NMF (input H)")
        if k == "auto":
            k = H.shape[0]
        if H.dtype != X.dtype and not (as_torch and X.dtype == torch.bfloat16):
            raise TypeError("H should have the same dtype as X. Got H.dtype = {}.".format(_dtype_name(H)))
        W = None  # filled with sqrt(X.mean()/k) below (SK:1228-1232)
    else:
        if W is not None or H is not None:
            warnings.warn("When init!='custom', provided W or H are ignored. Set  init='custom' to "
                          "use them as initialization.", RuntimeWarning)
        if k == "auto":
            k = n_features
        W, H = _initial_factors(X, int(k), init, random_state, device, as_torch, group, host_only=streamed,
                                init_device=init_device)
    k = int(k)
    if k > 16:
        raise ValueError(f"n_components={k} is not supported: the MI355X kernels handle 1..16.")
    if solver == "als" and k > 4:
        raise ValueError(f"n_components={k} is not supported by solver='als' (1..4).")
    if Mw is not None and k > 8:
        raise ValueError(f"n_components={k} is not supported by the weighted MU (1..8).")
    regs = _compute_regularization(n_samples, n_features, alpha_W, alpha_H, l1_ratio)
    return X, Mw, as_torch, streamed, k, W, H, regs


def _make_plan(X, Mw, k, regs, dev, *, solver="mu", sum_to_one=None, smoothness=0.0, group=None,
               streamed=False, memory_budget=None):
    """The plan (device state + launches) that runs the fit of X (all of it, or one shard)."""
    torch = _torch()
    from .solver import ALSPlan, MUPlan, WeightedMUPlan
    if streamed:  # §8 f3: X stays in host memory and streams through a memory_budget of HBM
        from .outofcore import StreamedMUPlan
        return StreamedMUPlan(X, k, regs[0], regs[2], regs[1], regs[3], group=group, device=dev,
                              memory_budget=memory_budget)
    Xd = X if _is_torch(X) else torch.from_numpy(np.ascontiguousarray(X))
    Xd = Xd.to(dev, non_blocking=False).contiguous()
    if Mw is not None:
        Md = (Mw if _is_torch(Mw) else torch.from_numpy(np.ascontiguousarray(Mw))).to(dev, torch.float32).contiguous()
        return WeightedMUPlan(Xd, Md, k, group=group)
    if solver == "als":
        return ALSPlan(Xd, k, sum_to_one=sum_to_one, smoothness=smoothness, group=group)
    return MUPlan(Xd, k, regs[0], regs[2], regs[1], regs[3], group=group)


def _start(plan, W, H, avg):
    """Load the starting factors; W None: the update_H=False start sqrt(X.mean()/k) (SK:1228-1232)."""
    torch = _torch()
    if W is None:
        plan.W.fill_(avg)
    else:
        plan.set_W(W if _is_torch(W) else torch.from_numpy(np.ascontiguousarray(W)))
    plan.set_H(H if _is_torch(H) else torch.from_numpy(np.ascontiguousarray(H)))


def _transform_start(X, as_torch, k):
    """sqrt(X.mean() / k) in X's dtype (SK:1228-1232)."""
    if as_torch:
        return float(_torch().sqrt(X.double().mean() / k))
    return float(np.sqrt(X.mean() / k))


def _fit_transform(X, W, H, n_components, init, update_H, tol, max_iter, alpha_W, alpha_H,
                   l1_ratio, random_state, verbose, device, group=None, return_plan=False,
                   normalise=None, solver="mu", sum_to_one=None, smoothness=0.0, weights=None,
                   memory_budget=None, init_device="auto"):
    """`_BaseNMF._fit_transform` for solver='mu' (SK:1638-1734) on the MI355X path."""
    torch = _torch()
    from .solver import run_mu

    X, Mw, as_torch, streamed, k, W, H, regs = _resolve(
        X, W, H, n_components, init, update_H, alpha_W, alpha_H, l1_ratio, random_state, device,
        group=group, solver=solver, normalise=normalise, weights=weights, memory_budget=memory_budget,
        init_device=init_device)
    dev = torch.device(device) if device is not None else (
        X.device if as_torch and X.device.type == "cuda" else torch.device("cuda", torch.cuda.current_device()))
    plan = _make_plan(X, Mw, k, regs, dev, solver=solver, sum_to_one=sum_to_one, smoothness=smoothness,
                      group=group, streamed=streamed, memory_budget=memory_budget)
    _start(plan, W, H, _transform_start(X, as_torch, k) if W is None else None)
    try:
        n_iter = run_mu(plan, max_iter=max_iter, tol=tol, update_H=update_H, verbose=verbose)
        if n_iter == max_iter and tol > 0:
            warnings.warn("Maximum number of iterations %d reached. Increase it to improve "
                          "convergence." % max_iter, ConvergenceWarning)
        if normalise is not None and update_H:
            plan.normalise(normalise)  # §8 a6: unit-norm basis rows, scales folded into W
        Wd, Hd = plan.W, plan.H()
        if return_plan:  # the caller releases the plan (NMF: after reconstruction_err_)
            return Wd, Hd, n_iter, plan, as_torch, X
        return _out(Wd, as_torch, X), _out(Hd, as_torch, X), n_iter
    except BaseException:
        _release(plan)
        raise
    finally:
        if not return_plan:
            _release(plan)


def _release(plan):
    """Unpin a streamed plan's host X and unmap exchange buffers now, not at garbage collection
    (a plan kept alive by a traceback would keep the caller's memory page-locked)."""
    rel = getattr(plan, "release", None)
    if rel is not None:
        rel()


def _out(t, as_torch, X):
    if as_torch:
        return t
    return t.detach().cpu().numpy().astype(X.dtype, copy=False)


def factorise(X, W=None, H=None, n_components="auto", *, init=None, update_H=True, solver="mu",
              beta_loss="frobenius", tol=1e-4, max_iter=200, alpha_W=0.0, alpha_H="same",
              l1_ratio=0.0, random_state=None, verbose=0, shuffle=False, device=None,
              normalise=None, sum_to_one=None, smoothness=0.0, weights=None, memory_budget=None,
              init_device="auto", devices=None):
    """Compute NMF X ≈ W·H with the multiplicative-update solver on an MI355X.

    Same signature, argument meaning, return value (W, H, n_iter) and errors as
    `sklearn.decomposition.non_negative_factorization` (SK:905-1131), except solver defaults to
    'mu' and takes 'mu' or 'als' (no 'cd').  `device` selects the HIP device (default: current).
    `normalise` ('l1' | 'l2' | 'max' | None, default None = sklearn's output): after the fit, every
    row of H is scaled to unit norm and the scale folded into W's column (W·H unchanged;
    SURVEY.md §8 a6).
    solver='als' selects the constrained ALS (k <= 4): per sample the exact
    non-negative least squares with a sum-to-one penalty of weight `sum_to_one` (δ; None = off),
    and per basis row the exact NNLS with a second-difference smoothness penalty `smoothness` (λ)
    — see oracle/als_ref.py for the precise objective.  tol / max_iter work as for 'mu'.
    `weights` (array of X's shape, >= 0; None = off) selects the weighted / masked MU (SURVEY.md
    §8(f) row 2, oracle/wmu_ref.py): the loss becomes Σ m·(x − wh)², so a weight 0 marks a missing
    value (give X any finite non-negative entry there) and 1/σ² an uncertainty weight; float32 X,
    k <= 8, no alpha regularisation; tol tests the weighted error.
    `memory_budget` (bytes; None = off): a host X (NumPy array, memory map or CPU tensor) larger
    than this is not copied to the GPU whole but streamed through HBM in row chunks every iteration
    (cnmf_amd.outofcore); same factors as the in-HBM fit up to fp summation order.
    `init_device` ('auto' | 'host' | 'gpu'): where init=None / 'nndsvd*' computes its SVD start —
    see `_initial_factors`; 'auto' reproduces sklearn's start for float32 X (host restatement) and
    runs the passes over X on the GPU for float64 X.
    `devices` (list of HIP device indices or torch devices; None = one device): split the rows
    over several GPUs driven from THIS process (cnmf_amd.multidevice): one stream and
    one persistent launch per device per stretch, the per-device [WᵀX | WᵀW] summed inside the
    launches over peer-mapped buffers.  Same factors as the one-device fit to fp64 summation order.
    """
    _validate_params(n_components, init, solver, beta_loss, tol, max_iter, alpha_W, alpha_H, l1_ratio)
    _validate_normalise(normalise)
    _validate_als(solver, alpha_W, alpha_H, sum_to_one, smoothness)
    _validate_init_device(init_device)
    if devices is not None:
        from .multidevice import factorise_devices
        return factorise_devices(X, W, H, n_components, devices=devices, init=init, update_H=update_H,
                                 solver=solver, tol=tol, max_iter=max_iter, alpha_W=alpha_W,
                                 alpha_H=alpha_H, l1_ratio=l1_ratio, random_state=random_state,
                                 verbose=verbose, normalise=normalise, sum_to_one=sum_to_one,
                                 smoothness=smoothness, weights=weights, init_device=init_device)
    return _fit_transform(X, W, H, n_components, init, update_H, tol, max_iter, alpha_W, alpha_H,
                          l1_ratio, random_state, verbose, device, normalise=normalise,
                          solver=solver, sum_to_one=sum_to_one, smoothness=smoothness,
                          weights=weights, memory_budget=memory_budget, init_device=init_device)


def _validate_normalise(normalise):
    if normalise not in (None, "l1", "l2", "max"):
        raise ValueError(f"The 'normalise' parameter must be a str among {{'l1', 'l2', 'max'}} or "
                         f"None. Got {normalise!r} instead.")


fit = factorise
non_negative_factorization = factorise


class NMF:
    """sklearn-shaped estimator (SK:1325-1763) on the MI355X MU path.

    Attributes after fit: components_, n_components_, n_iter_, reconstruction_err_,
    n_features_in_.
    """

    def __init__(self, n_components="auto", *, init=None, solver="mu", beta_loss="frobenius",
                 tol=1e-4, max_iter=200, random_state=None, alpha_W=0.0, alpha_H="same",
                 l1_ratio=0.0, verbose=0, shuffle=False, device=None, normalise=None,
                 sum_to_one=None, smoothness=0.0, memory_budget=None, init_device="auto"):
        self.n_components = n_components
        self.init_device = init_device
        self.memory_budget = memory_budget
        self.normalise = normalise
        self.sum_to_one = sum_to_one
        self.smoothness = smoothness
        self.init = init
        self.solver = solver
        self.beta_loss = beta_loss
        self.tol = tol
        self.max_iter = max_iter
        self.random_state = random_state
        self.alpha_W = alpha_W
        self.alpha_H = alpha_H
        self.l1_ratio = l1_ratio
        self.verbose = verbose
        self.shuffle = shuffle
        self.device = device

    def get_params(self, deep=True):
        return {k: getattr(self, k) for k in ("n_components", "init", "solver", "beta_loss", "tol",
                                              "max_iter", "random_state", "alpha_W", "alpha_H",
                                              "l1_ratio", "verbose", "shuffle", "device",
                                              "normalise", "sum_to_one", "smoothness", "memory_budget",
                                              "init_device")}

    def set_params(self, **params):
        for k, v in params.items():
            setattr(self, k, v)
        return self

    def _validate(self):
        _validate_params(self.n_components, self.init, self.solver, self.beta_loss, self.tol,
                         self.max_iter, self.alpha_W, self.alpha_H, self.l1_ratio)
        _validate_normalise(self.normalise)
        _validate_als(self.solver, self.alpha_W, self.alpha_H, self.sum_to_one, self.smoothness)
        _validate_init_device(self.init_device)

    def fit_transform(self, X, y=None, W=None, H=None, weights=None):
        """SK:1600-1636: learn the model, return W; sets reconstruction_err_ from the final W, H
        (the weighted error when `weights` is given: see `factorise`)."""
        self._validate()
        Wd, Hd, n_iter, plan, as_torch, Xc = _fit_transform(
            X, W, H, self.n_components, self.init, True, self.tol, self.max_iter, self.alpha_W,
            self.alpha_H, self.l1_ratio, self.random_state, self.verbose, self.device,
            return_plan=True, normalise=self.normalise, solver=self.solver,
            sum_to_one=self.sum_to_one, smoothness=self.smoothness, weights=weights,
            memory_budget=self.memory_budget, init_device=self.init_device)
        try:
            self.reconstruction_err_ = plan.frobenius_error()
            Wout = _out(Wd, as_torch, Xc)
            Hout = _out(Hd, as_torch, Xc)
        finally:
            _release(plan)
        self.n_components_ = int(Hd.shape[0])
        self.components_ = Hout
        self.n_iter_ = n_iter
        self.n_features_in_ = int(Xc.shape[1])
        return Wout

    def fit(self, X, y=None, **params):
        self.fit_transform(X, **params)
        return self

    def transform(self, X):
        """SK:1736-1763: solve for W with components_ fixed (update_H=False)."""
        if not hasattr(self, "components_"):
            raise ValueError("This NMF instance is not fitted yet. Call 'fit' with appropriate "
                             "arguments before using this estimator.")
        X = _check_X(X)
        _check_non_negative(X, "NMF (input X)")
        if X.shape[1] != self.n_features_in_:
            raise ValueError(f"X has {X.shape[1]} features, but NMF is expecting "
                             f"{self.n_features_in_} features as input.")
        W, _, _ = _fit_transform(X, None, self.components_, self.n_components_, self.init, False,
                                 self.tol, self.max_iter, self.alpha_W, self.alpha_H,
                                 self.l1_ratio, self.random_state, self.verbose, self.device,
                                 solver=self.solver, sum_to_one=self.sum_to_one,
                                 smoothness=self.smoothness, memory_budget=self.memory_budget)
        return W

    def inverse_transform(self, X=None, *, Xt=None):
        """W·H back in data space (SK `_BaseNMF.inverse_transform`)."""
        X = Xt if X is None else X
        if _is_torch(X):
            return X @ self.components_
        return np.asarray(X) @ self.components_
