"""GPU NNDSVD / NNDSVDA / NNDSVDAR initialisation.

sklearn's default init for k <= min(N, F) is NNDSVDA (SK:296-300) over
`randomized_svd(X, k, random_state)` (extmath.py:530-604).  The host restatement
(`cnmf_amd.init`) reproduces it bit for bit but costs seconds at cfg2's 1e6 x 81 (two passes of
X @ Q and X.T @ Q per power iteration, plus an N x 14 LU each time).  Here the passes over X run on
the GPU (libcnmf_hip.so, cnmf_init_*), and only F- and r-sized algebra stays on the host:

1. C = XᵀX and the column sums of X, fp64, ONE pass (cnmf_init_gram + cnmf_reduce_partials).
2. The range finder (extmath.py:287-357) in Gram form: sklearn alternates Q <- lu(X Q),
   Q <- lu(Xᵀ Q); only span(Q) enters the result, and span(Xᵀ X Z) = span(C Z).  So with the
   same Gaussian draw Ω (F x r, r = k + 10, drawn from the same RandomState and rounded to X's
   dtype as sklearn does) Z <- qr(C Z) for the same n_iter ('auto': 7 or 4).
3. The final Q = qr(X Z), B = Qᵀ X and svd(B) (extmath.py:576-590) without forming Q: with
   ZᵀCZ = V Λ Vᵀ, Q = X Z V Λ^-1/2 is an orthonormal basis of span(X Z), B = Λ^-1/2 Vᵀ Zᵀ C,
   and U = Q Uhat = X M with M = Z V Λ^-1/2 Uhat[:, :k] — ONE more pass (cnmf_init_xm).
   Directions with λ < 1e-14 λ_max (below fp64 resolution of the Gram form) are dropped.
4. svd_flip's u-based signs (extmath.py:900-953: the entry of largest |u| of each column, first
   occurrence) and the NNDSVD positive/negative part norms of U's columns: one pass over U
   (cnmf_init_stats); H and the choice of part per component on the host (SK:336-360).
5. W from U in one pass (cnmf_init_fill): |u| for j = 0, lbd · part / ‖part‖ otherwise,
   < eps -> 0, NNDSVDA's zeros -> X.mean() (SK:362-366).  NNDSVDAR's random fill of W's zeros in
   C order (SK:367-371) is done on the host copy of W (N x k), then W goes back to the device.

Agreement with sklearn (tests/test_gpu_init.py, tests/golden/init_*.npz): the result is the same
randomized SVD up to floating point; with fp64 X the GPU init matches sklearn to ~1e-9 when the
k-th singular value of X is above ~1e-6 of the first (the Gram form squares the condition of the
trailing directions; components below X's rounding level are noise in any implementation).  With
fp32 X sklearn computes the whole SVD in fp32, so the two differ at fp32 rounding (~1e-6).
"""
from __future__ import annotations

from math import sqrt

import numpy as np
import torch
from scipy import linalg

from . import _lib
from ._lib import check
from .init import _check_random_state

__all__ = ["gpu_init_eligible", "initialize_nmf_gpu", "GPU_INIT_MAX_FEATURES", "GPU_INIT_MAX_K"]

GPU_INIT_MAX_FEATURES = 96
GPU_INIT_MAX_K = 16
_XDT = {torch.float32: _lib.F32, torch.float64: _lib.F64, torch.bfloat16: _lib.BF16}


def gpu_init_eligible(n_samples: int, n_features: int, k: int, init, dtype) -> bool:
    """The GPU path serves the NNDSVD family for N >= F (sklearn's non-transposed branch),
    F <= 96, k <= 16, fp32 / fp64 / bf16 X."""
    return (init in ("nndsvd", "nndsvda", "nndsvdar") and n_samples >= n_features
            and n_features <= GPU_INIT_MAX_FEATURES and 1 <= k <= min(GPU_INIT_MAX_K, n_features)
            and dtype in _XDT)


def _ptr(t):
    return t.data_ptr()


def _reduce(lib, parts, n_rows, n_out, dev, stream):
    out = torch.empty(n_out, dtype=torch.float64, device=dev)
    stage = torch.zeros(int(lib.cnmf_stage_doubles(n_out)), dtype=torch.float64, device=dev)
    counter = torch.zeros(int(lib.cnmf_counter_words()), dtype=torch.int32, device=dev)
    check(lib.cnmf_reduce_partials(_ptr(parts), n_rows, n_out, _ptr(stage), _ptr(counter), _ptr(out),
                                   stream), "cnmf_reduce_partials")
    return out


def initialize_nmf_gpu(X: torch.Tensor, n_components: int, init: str = "nndsvda", eps: float = 1e-6,
                       random_state=None):
    """(W, H) for the NNDSVD family from X (N x F, on a HIP device).  W: device tensor of X's
    compute dtype (fp64 for fp64 X, else fp32); H: NumPy array of the same dtype."""
    if X.device.type != "cuda":
        raise _lib.HipLibraryError("initialize_nmf_gpu needs X on a HIP device")
    N, F = (int(v) for v in X.shape)
    k = int(n_components)
    if not gpu_init_eligible(N, F, k, init, X.dtype):
        raise ValueError(f"GPU init does not serve init={init!r} for X {N}x{F} {X.dtype} k={k}")
    lib = _lib.load()
    dev = X.device
    X = X.contiguous()
    xdt = _XDT[X.dtype]
    np_dt = np.float64 if X.dtype == torch.float64 else np.float32
    with torch.cuda.device(dev):
        stream = torch.cuda.current_stream(dev).cuda_stream
        # 1. C = XᵀX and the column sums (one pass over X)
        g = int(check(lib.cnmf_init_gram_rows(N), "cnmf_init_gram_rows"))
        n_out = F * F + F
        parts = torch.empty((g, n_out), dtype=torch.float64, device=dev)
        check(lib.cnmf_init_gram(_ptr(X), xdt, N, F, _ptr(parts), g, stream), "cnmf_init_gram")
        o = _reduce(lib, parts, g, n_out, dev, stream).cpu().numpy()
        del parts
        C = o[:F * F].reshape(F, F)
        C = 0.5 * (C + C.T)
        avg = float(o[F * F:].sum() / (N * F))  # X.mean() (sklearn: in X's dtype)

        # 2. the range finder in Gram form (extmath.py:287-357), same draw as sklearn
        rs = _check_random_state(random_state)
        r = k + 10
        n_iter = 7 if k < 0.1 * min(N, F) else 4
        Om = rs.normal(size=(F, r))
        if np_dt == np.float32:
            Om = Om.astype(np.float32)
        Z = Om.astype(np.float64)
        for _ in range(n_iter):
            Z, _ = linalg.qr(C @ Z, mode="economic")
        # 3. Q = X Z V Λ^-1/2 (never formed), B = Qᵀ X, svd(B), U = X M
        lam, Vy = linalg.eigh(Z.T @ C @ Z)
        keep = lam > lam.max() * 1e-14
        T = Vy[:, keep] / np.sqrt(lam[keep])
        B = T.T @ (Z.T @ C)
        Uhat, s, Vt = linalg.svd(B, full_matrices=False, lapack_driver="gesdd")
        kk = min(k, Uhat.shape[1])
        M = np.zeros((F, k))
        M[:, :kk] = Z @ T @ Uhat[:, :kk]
        S = np.zeros(k)
        S[:kk] = s[:kk]
        V = np.zeros((k, F))
        V[:kk] = Vt[:kk]
        Md = torch.from_numpy(np.ascontiguousarray(M)).to(dev)
        U = torch.empty((N, k), dtype=torch.float64, device=dev)
        check(lib.cnmf_init_xm(_ptr(X), xdt, N, F, k, _ptr(Md), _ptr(U), stream), "cnmf_init_xm")

        # 4. signs (svd_flip, u-based) and the part norms of U's columns
        gs = int(check(lib.cnmf_init_stats_rows(N), "cnmf_init_stats_rows"))
        st = torch.empty((gs, k * 5), dtype=torch.float64, device=dev)
        check(lib.cnmf_init_stats(_ptr(U), N, k, _ptr(st), gs, stream), "cnmf_init_stats")
        st = st.cpu().numpy().reshape(gs, k, 5)
        sp = st[:, :, 0].sum(axis=0)
        sn = st[:, :, 1].sum(axis=0)
        sign = np.ones(k)
        for j in range(k):
            best, val, row = -1.0, 0.0, 0.0
            for b in range(gs):  # workgroups in row order; ties: the lower row (np.argmax)
                m, v, i = st[b, j, 2], st[b, j, 3], st[b, j, 4]
                if m > best or (m == best and i < row):
                    best, val, row = m, v, i
            sign[j] = np.sign(val) if val != 0 else 1.0
        V = V * sign[:, None]
        pos = np.where(sign > 0, sp, sn)  # ‖max(sign·u, 0)‖²
        neg = np.where(sign > 0, sn, sp)

        # NNDSVD (SK:336-360): per component the part of (u, v) with the larger norm product
        H = np.zeros((k, F))
        coef = np.zeros(k)
        part = np.zeros(k, dtype=np.int32)
        coef[0] = sqrt(S[0])
        H[0] = sqrt(S[0]) * np.abs(V[0])
        for j in range(1, k):
            y = V[j]
            y_p, y_n = np.maximum(y, 0), np.abs(np.minimum(y, 0))
            x_p_nrm, x_n_nrm = sqrt(pos[j]), sqrt(neg[j])
            y_p_nrm, y_n_nrm = sqrt(float(np.dot(y_p, y_p))), sqrt(float(np.dot(y_n, y_n)))
            m_p, m_n = x_p_nrm * y_p_nrm, x_n_nrm * y_n_nrm
            if m_p > m_n:
                nrm, v, sigma, part[j] = x_p_nrm, y_p / y_p_nrm, m_p, 1
            else:
                nrm, v, sigma, part[j] = x_n_nrm, y_n / y_n_nrm, m_n, 2
            lbd = sqrt(S[j] * sigma)
            coef[j] = lbd / nrm if nrm > 0 else 0.0
            H[j] = lbd * v
        H = H.astype(np_dt)
        H[H < eps] = 0

        # 5. W (one pass over U), the NNDSVDA / NNDSVDAR fills
        wdt = _lib.F64 if np_dt == np.float64 else _lib.F32
        W = torch.empty((N, k), dtype=torch.float64 if np_dt == np.float64 else torch.float32, device=dev)
        fill = avg if init == "nndsvda" else 0.0
        cd = torch.from_numpy(coef).to(dev)
        pd = torch.from_numpy(part).to(dev)
        sd = torch.from_numpy(sign).to(dev)
        check(lib.cnmf_init_fill(_ptr(U), N, k, _ptr(cd), _ptr(pd), _ptr(sd), float(eps), float(fill),
                                 _ptr(W), wdt, stream), "cnmf_init_fill")
        del U
        avg_x = np_dt(avg)
        if init == "nndsvda":
            H[H == 0] = avg_x
        elif init == "nndsvdar":
            rng = _check_random_state(random_state)
            Wh = W.cpu().numpy()
            Wh[Wh == 0] = abs(avg_x * rng.standard_normal(size=len(Wh[Wh == 0])) / 100)
            H[H == 0] = abs(avg_x * rng.standard_normal(size=len(H[H == 0])) / 100)
            W.copy_(torch.from_numpy(Wh))
        torch.cuda.current_stream(dev).synchronize()
    return W, H
