"""cfg4-shaped (bf16 X, F = 300, k = 16) agreement between the persistent launch (layout 6) and the
per-iteration launches (layout 4) over 40 iterations, and each against the fp64 oracle on the
bf16-rounded X — the numbers behind tests/test_gpu_cfg4_persistent.py's bars, printed for a library
(CNMF_HIP_LIB) so that two kernel forms can be compared on one box (round 6: H in two bf16 terms).

    python tools/cfg4_layout_probe.py [n_tiles ...]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))


def main(tiles):
    import torch
    from cnmf_amd.solver import MUPlan
    from cnmf_amd.synthetic import iop_spectra, random_init
    from golden_io import rel_fro
    from oracle import mu_ref
    for n_tiles in tiles:
        X32 = iop_spectra(64 * n_tiles, 300, seed=n_tiles, dtype=np.float32)
        Xb = torch.from_numpy(X32).to(torch.bfloat16)
        Xr = Xb.float().numpy()
        W0, H0 = random_init(Xr, 16, 42)
        out = {}
        for lay in (6, 4):
            p = MUPlan(Xb.cuda(), 16)
            p.set_layout(lay)
            p.set_W(torch.from_numpy(W0))
            p.set_H(torch.from_numpy(H0))
            p.iterate(40)
            torch.cuda.synchronize()
            out[lay] = (p.W.cpu().numpy(), p.H64.cpu().numpy())
        Wr, Hr, _ = mu_ref.mu_fit(Xr.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                                  max_iter=40, tol=0.0)
        print(f"n_tiles {n_tiles}: layout 6 vs 4 W {rel_fro(out[6][0], out[4][0]):.2e} H {rel_fro(out[6][1], out[4][1]):.2e}; "
              f"vs oracle W {rel_fro(out[4][0], Wr):.2e} H {rel_fro(out[4][1], Hr):.2e}", flush=True)


if __name__ == "__main__":
    main([int(a) for a in sys.argv[1:]] or [50, 200, 3000])
