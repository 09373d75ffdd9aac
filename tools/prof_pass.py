"""Minimal launch driver for rocprofv3 counter collection: N launches of the fused pass (and the
reduce/update tail) on the cfg2 shape, nothing else on the GPU."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--features", type=int, default=81)
    ap.add_argument("--k", type=int, default=4)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"])
    ap.add_argument("--solver", default="mu", choices=["mu", "als"],
                    help="als: the persistent constrained ALS (sum_to_one 1, smoothness 0.5)")
    ap.add_argument("--layout", type=int, default=0, help="the persistent launch's layout (include/cnmf_hip.h)")
    a = ap.parse_args()
    import torch
    from cnmf_amd.solver import MUPlan
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(a.rows, a.features, seed=0, dtype=np.float32)
    W0, H0 = random_init(X, a.k, 42)
    Xd = torch.from_numpy(X).cuda()
    if a.dtype == "bf16":
        Xd = Xd.to(torch.bfloat16)
    if a.solver == "als":
        from cnmf_amd.solver import ALSPlan
        plan = ALSPlan(Xd, a.k, sum_to_one=1.0, smoothness=0.5)
    else:
        plan = MUPlan(Xd, a.k)
        plan.layout = a.layout
    plan.set_W(torch.from_numpy(W0))
    plan.set_H(torch.from_numpy(H0))
    plan.iterate(a.iters)
    torch.cuda.synchronize()
    print("done", plan.n_parts, flush=True)


if __name__ == "__main__":
    main()
