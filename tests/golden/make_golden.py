"""Generate the committed golden vectors under tests/golden/ by running scikit-learn itself.

Run in the BUILD container only (sklearn 1.7.2 is importable there; it is the MU implementation
the reference declares as a dependency, /root/reference/setup.py:26,30).  The GPU box never runs
this script: it only reads the .npz files it writes.  Each case stores its inputs (X, W0, H0 or the
init recipe), the call's keyword arguments, and sklearn's outputs (W, H, n_iter).

    python tests/golden/make_golden.py         # rewrites tests/golden/*.npz + MANIFEST.json
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from cnmf_amd.synthetic import iop_spectra, random_init  # noqa: E402


def _bf16_round(a):
    """Round-to-nearest-even fp32 -> bf16 -> fp32 (the values a bf16 X actually holds)."""
    u = np.ascontiguousarray(a, dtype=np.float32).view(np.uint32).astype(np.uint64)
    u = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return u.astype(np.uint32).view(np.float32)


def cases():
    """(name, X, W0, H0, kwargs).  W0/H0 None => sklearn does its own init from kwargs."""
    out = []
    # cfg1 (BASELINE.json configs[0]): 1000x81 IOP, k=4, 200 iters, fixed-iteration (tol=0)
    for dt in (np.float64, np.float32):
        X = iop_spectra(1000, 81, seed=0, dtype=dt)
        W0, H0 = random_init(X, 4, 42)
        out.append((f"cfg1_{np.dtype(dt).name}", X, W0, H0,
                    dict(n_components=4, init="custom", tol=0.0, max_iter=200)))
    # k=8 (cfg3 shape class), 2048x81, 50 iters
    X = iop_spectra(2048, 81, seed=1, dtype=np.float32)
    W0, H0 = random_init(X, 8, 42)
    out.append(("k8_float32", X, W0, H0, dict(n_components=8, init="custom", tol=0.0, max_iter=50)))
    # F=300, k=16 on bf16-representable values (cfg4 shape class), 20 iters
    X = _bf16_round(iop_spectra(512, 300, seed=2, dtype=np.float32))
    W0, H0 = random_init(X, 16, 42)
    out.append(("f300k16_bf16vals", X, W0, H0,
                dict(n_components=16, init="custom", tol=0.0, max_iter=20)))
    # sklearn test_nmf_multiplicative_update_sparse shapes (SKT:502-577): 20x10, k=5, RandomState(1337)
    rng = np.random.mtrand.RandomState(1337)
    Xs = np.abs(rng.randn(20, 10))
    for name, kw in [("sk20x10_plain", dict(alpha_W=0.0, l1_ratio=0.0)),
                     ("sk20x10_l1l2", dict(alpha_W=0.5, l1_ratio=0.5)),
                     ("sk20x10_l2", dict(alpha_W=0.3, alpha_H=0.1, l1_ratio=0.0)),
                     ("sk20x10_l1", dict(alpha_W=0.2, l1_ratio=1.0))]:
        out.append((name, Xs, None, None,
                    dict(n_components=5, init="random", random_state=42, tol=0.0, max_iter=20, **kw)))
    # tol > 0: iteration-count semantics (SK:872-884), fp64 and fp32
    for dt in (np.float64, np.float32):
        X = iop_spectra(300, 81, seed=3, dtype=dt)
        W0, H0 = random_init(X, 4, 7)
        out.append((f"tol_{np.dtype(dt).name}", X, W0, H0,
                    dict(n_components=4, init="custom", tol=1e-3, max_iter=500)))
    # zero rows and zero columns exercise the EPSILON branch (SK:620, SK:706)
    X = iop_spectra(257, 81, seed=4, dtype=np.float32)
    X[[0, 5, 100, 256]] = 0.0
    X[:, [3, 40]] = 0.0
    W0, H0 = random_init(X, 4, 11)
    out.append(("zeros_float32", X, W0, H0, dict(n_components=4, init="custom", tol=0.0, max_iter=30)))
    # odd shapes: N not a multiple of the 64-sample tile, k not a multiple of 4
    X = iop_spectra(333, 81, seed=5, dtype=np.float32)
    W0, H0 = random_init(X, 5, 12)
    out.append(("ragged_k5_float32", X, W0, H0, dict(n_components=5, init="custom", tol=0.0, max_iter=40)))
    X = iop_spectra(130, 17, seed=6, dtype=np.float64)
    W0, H0 = random_init(X, 3, 13)
    out.append(("ragged_f17_float64", X, W0, H0, dict(n_components=3, init="custom", tol=0.0, max_iter=40)))
    # init='random' handled inside sklearn (our host init must reproduce the draws)
    X = iop_spectra(400, 81, seed=7, dtype=np.float32)
    out.append(("initrandom_float32", X, None, None,
                dict(n_components=4, init="random", random_state=0, tol=0.0, max_iter=25)))
    # update_H=False (transform path): H fixed, W starts at sqrt(mean/k) (SK:1221-1232)
    X = iop_spectra(500, 81, seed=8, dtype=np.float32)
    _, H0 = random_init(X, 4, 21)
    out.append(("transform_float32", X, None, H0,
                dict(n_components=4, init="custom", update_H=False, tol=0.0, max_iter=60)))
    # regularised IOP case in fp32
    X = iop_spectra(700, 81, seed=9, dtype=np.float32)
    W0, H0 = random_init(X, 4, 5)
    out.append(("reg_float32", X, W0, H0,
                dict(n_components=4, init="custom", alpha_W=1e-3, alpha_H=2e-4, l1_ratio=0.3,
                     tol=0.0, max_iter=50)))
    return out


def init_cases():
    """(name, X, kwargs) for sklearn's _initialize_nmf (SK:221-373): the NNDSVD family over
    randomized_svd (extmath.py:530-604), fp64 and fp32, plus init=None's default (nndsvda)."""
    out = []
    X64 = iop_spectra(1024, 81, seed=10, dtype=np.float64)
    for init in ("nndsvd", "nndsvda", "nndsvdar"):
        out.append((f"init_{init}_float64", X64, dict(n_components=4, init=init, random_state=0)))
    X32 = iop_spectra(1024, 81, seed=11, dtype=np.float32)
    for init in ("nndsvda", "nndsvdar"):
        out.append((f"init_{init}_float32", X32, dict(n_components=4, init=init, random_state=0)))
    Xr = np.random.RandomState(3).rand(1024, 60)  # well conditioned: every component is signal
    out.append(("init_rand_k8_float64", Xr, dict(n_components=8, init="nndsvda", random_state=1)))
    Xd = iop_spectra(1024, 81, seed=12, dtype=np.float32)
    out.append(("init_default_float32", Xd, dict(n_components=4, init=None, random_state=2)))
    return out


def main_init(manifest):
    from sklearn.decomposition._nmf import _initialize_nmf
    manifest["init_generator"] = "sklearn.decomposition._nmf._initialize_nmf"
    manifest["init_cases"] = {}
    for name, X, kw in init_cases():
        W, H = _initialize_nmf(X, kw["n_components"], init=kw["init"], random_state=kw["random_state"])
        arrays = {"X": X, "W": W, "H": H, "kwargs": np.array(json.dumps(kw))}
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **arrays)
        with open(path, "rb") as f:
            digest = hashlib.sha256(f.read()).hexdigest()
        manifest["init_cases"][name] = {"sha256": digest, "kwargs": kw, "shape": list(X.shape),
                                        "dtype": str(X.dtype)}
        print(f"{name:24s} {str(X.shape):14s} {str(X.dtype):8s} init={kw['init']}")


def tall_cases():
    """(name, seed, n_rows, kwargs): sklearn's DEFAULT fit (init=None -> nndsvda over randomized_svd,
    tol=1e-4, max_iter=200) on tall fp32 X — the path cnmf's API routes X of >= 65,536 rows through
    (VERDICT r2).  X is NOT stored: the test regenerates it from iop_spectra(seed) and checks its
    sha256; only sklearn's start (_initialize_nmf) and result are stored."""
    return [("tall_default_float32", 13, 65536, dict(n_components=4, random_state=0)),
            # the same default start with a tolerance that stops early (n_iter semantics, SK:872-884)
            ("tall_default_tol_float32", 14, 65536, dict(n_components=4, random_state=0, tol=1e-3,
                                                         max_iter=500))]


def main_tall(manifest):
    from sklearn.decomposition import non_negative_factorization
    from sklearn.decomposition._nmf import _initialize_nmf
    manifest["tall_cases"] = {}
    for name, seed, n, kw in tall_cases():
        X = iop_spectra(n, 81, seed=seed, dtype=np.float32)
        W0, H0 = _initialize_nmf(X, kw["n_components"], init=None, random_state=kw["random_state"])
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            W, H, n_iter = non_negative_factorization(X, solver="mu", **kw)
        x_sha = hashlib.sha256(np.ascontiguousarray(X).tobytes()).hexdigest()
        arrays = {"W_init": W0, "H_init": H0, "W": W, "H": H, "n_iter": np.int64(n_iter),
                  "seed": np.int64(seed), "n_rows": np.int64(n), "x_sha256": np.array(x_sha),
                  "kwargs": np.array(json.dumps(kw))}
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **arrays)
        with open(path, "rb") as f:
            digest = hashlib.sha256(f.read()).hexdigest()
        manifest["tall_cases"][name] = {"sha256": digest, "kwargs": kw, "n_iter": int(n_iter),
                                        "seed": seed, "shape": [n, 81], "dtype": "float32",
                                        "x_sha256": x_sha}
        print(f"{name:24s} {(n, 81)} float32 default init, n_iter={n_iter}")


def main():
    from sklearn.decomposition import non_negative_factorization
    import sklearn

    manifest = {"generator": "sklearn.decomposition.non_negative_factorization(solver='mu')",
                "sklearn_version": sklearn.__version__, "numpy_version": np.__version__,
                "cases": {}}
    for name, X, W0, H0, kw in cases():
        kw = dict(kw)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            W, H, n_iter = non_negative_factorization(
                X, None if W0 is None else W0.copy(), None if H0 is None else H0.copy(),
                solver="mu", **kw)
        arrays = {"X": X, "W": W, "H": H, "n_iter": np.int64(n_iter)}
        if W0 is not None:
            arrays["W0"] = W0
        if H0 is not None:
            arrays["H0"] = H0
        arrays["kwargs"] = np.array(json.dumps(kw))
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **arrays)
        with open(path, "rb") as f:
            digest = hashlib.sha256(f.read()).hexdigest()
        manifest["cases"][name] = {"sha256": digest, "kwargs": kw, "n_iter": int(n_iter),
                                   "shape": list(X.shape), "dtype": str(X.dtype)}
        print(f"{name:24s} {str(X.shape):14s} {str(X.dtype):8s} n_iter={n_iter}")
    main_init(manifest)
    main_tall(manifest)
    with open(os.path.join(HERE, "MANIFEST.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


def main_only_tall():
    """Add / refresh the tall default-init cases without rewriting the others."""
    with open(os.path.join(HERE, "MANIFEST.json")) as f:
        manifest = json.load(f)
    main_tall(manifest)
    with open(os.path.join(HERE, "MANIFEST.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    if "--only-tall" in sys.argv:
        main_only_tall()
    else:
        main()
