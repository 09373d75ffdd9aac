"""Diagnostic: repeatability of the wave-tile persistent launch across split launches.
For each case: one launch of n iterations vs a split (a + b), and two identical single launches;
prints the number of differing W rows, which tile positions they sit at, and the max difference."""
import sys
import numpy as np
import torch

sys.path.insert(0, ".")
from cnmf_amd.solver import MUPlan
from cnmf_amd.synthetic import iop_spectra, random_init


def plan(X, W0, H0):
    p = MUPlan(X, W0.shape[1])
    p.set_W(torch.from_numpy(W0))
    p.set_H(torch.from_numpy(H0))
    return p


def report(tag, a, b, k):
    dW = (a.W - b.W).abs()
    rows = torch.nonzero(dW.amax(dim=1) > 0).flatten().cpu().numpy()
    dH = float((a.H64 - b.H64).abs().max())
    tsw = 64 // k
    tiles = np.unique(rows // tsw)
    print(f"{tag}: rows differing {len(rows)} tiles {len(tiles)} maxdW {float(dW.max()):.3e} maxdH {dH:.3e} "
          f"first tiles {tiles[:12].tolist()}", flush=True)


for N, k, its in [(1_250_000, 8, (1, 1)), (1_250_000, 8, (2, 3)), (200_000, 8, (2, 3)), (2_000_000, 4, (2, 3))]:
    X = iop_spectra(N, 81, seed=3, dtype=np.float32)
    W0, H0 = random_init(X, k, 42)
    Xd = torch.from_numpy(X).cuda()
    n = sum(its)
    a, b, c = plan(Xd, W0, H0), plan(Xd, W0, H0), plan(Xd, W0, H0)
    print(f"N={N} k={k} persistent={a.persistent}", flush=True)
    a.iterate(n)
    for m in its:
        b.iterate(m)
    c.iterate(n)
    torch.cuda.synchronize()
    a.check_sync_error()
    report(f"  single vs split {its}", a, b, k)
    report(f"  single vs single", a, c, k)
    # one iteration per launch, repeated
    d, e = plan(Xd, W0, H0), plan(Xd, W0, H0)
    d.iterate(1)
    e.iterate(1)
    torch.cuda.synchronize()
    report("  1 iter vs 1 iter", d, e, k)
