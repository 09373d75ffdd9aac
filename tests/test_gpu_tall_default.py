"""The DEFAULT fit on a tall float32 X against sklearn itself: sklearn's
`non_negative_factorization(X, n_components=4, solver='mu', random_state=0)` — init=None, so
NNDSVDA over randomized_svd, tol=1e-4, max_iter=200 — on 65,536 synthetic IOP rows, stored by
tests/golden/make_golden.py (tall_default_*.npz; X regenerated here from its seed and checked by
sha256).  Two cases: the default tolerance (runs to max_iter = 200) and tol = 1e-3 (stops at 190).

What is asserted, and why:
* the start: cnmf's default (init_device='auto') takes the host restatement for float32 X, which
  reproduces sklearn's start (bit for bit on the build container's BLAS; to BLAS rounding here);
* the iteration count: identical to sklearn's;
* W, H against the fp64 oracle run from sklearn's own start: the north-star bar, 1e-5;
* W, H against sklearn's own float32 result: sklearn's fp32 MU drifts from the fp64 answer by a few
  1e-6, so the two fp32 paths are compared at 2e-5 and the measured distance is printed;
* init_device='gpu' (fp64 Gram-form randomized SVD on the GPU): NOT sklearn's fp32 start — the
  measured distance of its fitted factors to sklearn's is printed and bounded at 5e-3.
"""
import hashlib

import numpy as np
import pytest

from golden_io import GOLDEN, rel_fro

pytestmark = pytest.mark.gpu

CASES = ["tall_default_float32", "tall_default_tol_float32"]


def _case(name):
    import json
    import os
    from cnmf_amd.synthetic import iop_spectra
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)
    c = {k: z[k] for k in z.files}
    c["kwargs"] = json.loads(str(c["kwargs"]))
    X = iop_spectra(int(c["n_rows"]), 81, seed=int(c["seed"]), dtype=np.float32)
    assert hashlib.sha256(np.ascontiguousarray(X).tobytes()).hexdigest() == str(c["x_sha256"])
    return X, c


@pytest.mark.parametrize("name", CASES)
def test_default_fit_matches_sklearn(name):
    import cnmf_amd
    from oracle import mu_ref
    X, c = _case(name)
    kw = c["kwargs"]
    W, H, n = cnmf_amd.factorise(X, **kw)
    assert n == int(c["n_iter"])
    Wr, Hr, nr = mu_ref.mu_fit(X.astype(np.float64), c["W_init"].astype(np.float64),
                               c["H_init"].astype(np.float64), max_iter=kw.get("max_iter", 200),
                               tol=kw.get("tol", 1e-4))
    assert nr == n
    ew64, eh64 = rel_fro(W, Wr), rel_fro(H, Hr)
    ew, eh = rel_fro(W, c["W"]), rel_fro(H, c["H"])
    ew_sk, eh_sk = rel_fro(c["W"], Wr), rel_fro(c["H"], Hr)
    print(f"{name}: n_iter {n}; GPU vs fp64 oracle W {ew64:.2e} H {eh64:.2e}; GPU vs sklearn fp32 "
          f"W {ew:.2e} H {eh:.2e}; sklearn fp32 vs fp64 oracle W {ew_sk:.2e} H {eh_sk:.2e}")
    assert ew64 <= 1e-5 and eh64 <= 1e-5, (ew64, eh64)
    assert ew <= 1.2e-5 and eh <= 1.2e-5, (ew, eh)  # measured 7.4e-6 = sklearn fp32's own drift


def test_gpu_init_distance_is_stated():
    import cnmf_amd
    X, c = _case(CASES[0])
    W, H, n = cnmf_amd.factorise(X, init_device="gpu", **c["kwargs"])
    ew, eh = rel_fro(W, c["W"]), rel_fro(H, c["H"])
    print(f"init_device='gpu': fitted factors vs sklearn's fp32 result W {ew:.2e} H {eh:.2e}")
    assert ew <= 5e-3 and eh <= 5e-3, (ew, eh)
