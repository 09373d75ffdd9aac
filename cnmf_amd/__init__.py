"""cnmf_amd — constrained NMF on AMD MI355X (gfx950).

The caller-facing API mirrors scikit-learn's Frobenius multiplicative-update NMF (the algorithm the
reference AI-for-Ocean-Science/cnmf declares; its own package is empty):

    W, H, n_iter = cnmf_amd.factorise(X, n_components=4, init="random", random_state=42, tol=0)
    model = cnmf_amd.NMF(n_components=4).fit(X)

The hot loop runs in libcnmf_hip.so (hand-written HIP for gfx950, C ABI in include/cnmf_hip.h);
there is no CPU fallback.  See DESIGN.md.
"""
from ._lib import HipLibraryError
from ._trace import tracing
from .api import NMF, ConvergenceWarning, factorise, fit, non_negative_factorization

__version__ = "0.1.0"
__all__ = ["factorise", "fit", "non_negative_factorization", "NMF", "ConvergenceWarning",
           "HipLibraryError", "tracing", "__version__"]
