"""Time the persistent layouts (1 = pairs, 3 = floating tiles at several fractions) on a few shapes.

    python tools/dyn_probe.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from cnmf_amd import _lib
    from cnmf_amd.solver import MUPlan
    from cnmf_amd.synthetic import iop_spectra, random_init
    lib = _lib.load()
    for n_tiles in (4096, 15625):
        X = iop_spectra(64 * n_tiles, 81, seed=0, dtype=np.float32)
        W0, H0 = random_init(X, 4, 42)
        plan = MUPlan(torch.from_numpy(X).cuda(), 4)
        plan.set_W(torch.from_numpy(W0))
        plan.set_H(torch.from_numpy(H0))
        plan.iterate(1000)
        torch.cuda.synchronize()
        for v, frac in ((1, None), (3, 1.0), (3, 0.95), (3, 0.9), (3, 0.8), (1, None)):
            lib.cnmf_set_persist_variant(v)
            if frac:
                lib.cnmf_set_persist_dyn_frac(frac)
            ts = []
            for _ in range(3):
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                ev[0].record()
                plan.iterate(200)
                ev[1].record()
                torch.cuda.synchronize()
                plan.check_sync_error()
                ts.append(ev[0].elapsed_time(ev[1]) * 1e3 / 200)
            print(f"tiles {n_tiles} variant {v} frac {frac}: {min(ts):.2f} us/it ({[round(t, 2) for t in ts]})",
                  flush=True)
        lib.cnmf_set_persist_variant(1)
        del plan


if __name__ == "__main__":
    main()
