"""Bit-level probe of the persistent weighted-MU / ALS launches (round 6 debugging aid): saves W, H after
15 iterations of the single-GPU launch, and (--multi) of the self-exchange launch as 15 and as 6 + 9
iterations, for tools/npz_bits_cmp.py.

    CNMF_HIP_LIB=<lib> python tools/wmu_bits_probe.py out.npz [--multi]
"""
import os
import socket
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(out, multi):
    import torch
    from cnmf_amd.solver import ALSPlan, WeightedMUPlan
    from cnmf_amd.synthetic import iop_spectra, random_init
    N = 64 * 700
    X = iop_spectra(N, 81, seed=3, dtype=np.float32)
    rng = np.random.default_rng(3)
    M = (rng.uniform(0.2, 2.0, X.shape) * (rng.random(X.shape) >= 0.3)).astype(np.float32)
    W0, H0 = random_init(X, 4, 42)
    res = {}
    group = None
    if multi:
        import torch.distributed as dist
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
        group = dist.group.WORLD
    for name, split, g in (("single", (15,), None), ("multi15", (15,), group), ("multi6_9", (6, 9), group)):
        if g is None and name != "single":
            continue
        p = WeightedMUPlan(torch.from_numpy(X).cuda(), torch.from_numpy(M).cuda(), 4, group=g)
        p.set_W(torch.from_numpy(W0))
        p.set_H(torch.from_numpy(H0))
        if g is not None:
            p.enable_exchange()
        for n in split:
            p.iterate(n)
        p.check_sync_error()
        torch.cuda.synchronize()
        res[name + "_W"], res[name + "_H"], res[name + "_AD"] = p.W.cpu().numpy(), p.H64.cpu().numpy(), p.AD.cpu().numpy()
        if g is not None:
            p.release()
    a = ALSPlan(torch.from_numpy(X).cuda(), 4, sum_to_one=1.0, smoothness=0.5)
    a.set_W(torch.from_numpy(W0))
    a.set_H(torch.from_numpy(H0))
    a.iterate(15)
    a.check_sync_error()
    torch.cuda.synchronize()
    res["als_W"], res["als_H"] = a.W.cpu().numpy(), a.H64.cpu().numpy()
    np.savez(out, **res)
    print("saved", out, sorted(res))


if __name__ == "__main__":
    main(sys.argv[1], "--multi" in sys.argv)
