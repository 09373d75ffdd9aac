"""Diagnostic: µs per MU iteration of the persistent cfg2 launch for several rotated-window sizes
(CNMF_ROT_MB, read by the library at every launch) and persistent layouts.

    python tools/rot_probe.py [--mb 0,120,160,200,240] [--variants 1,2] [--iters 500] [--rounds 2]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", default="0,120,160,200,240")
    ap.add_argument("--variants", default="1,2")
    ap.add_argument("--iters", type=int, default=500)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--rows", type=int, default=1_000_000)
    args = ap.parse_args()
    import numpy as np
    import torch
    from cnmf_amd.solver import MUPlan
    from cnmf_amd.synthetic import iop_spectra, random_init

    X = iop_spectra(args.rows, 81, seed=0, dtype=np.float32)
    W0, H0 = random_init(X, 4, 42)
    plan = MUPlan(torch.from_numpy(X).cuda(), 4)
    plan.set_W(torch.from_numpy(W0))
    plan.set_H(torch.from_numpy(H0).cuda())
    plan.iterate(1500)  # clocks up
    torch.cuda.synchronize()
    mbs = [float(v) for v in args.mb.split(",")]
    variants = [int(v) for v in args.variants.split(",")]
    res = {}
    st = torch.cuda.current_stream()
    for _ in range(args.rounds):
        for v in variants:
            plan.lib.cnmf_set_persist_variant(v)
            for mb in mbs:
                os.environ["CNMF_ROT_MB"] = str(mb)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                plan.iterate(args.iters)
                e1.record(st)
                torch.cuda.synchronize()
                plan.check_sync_error()
                us = e0.elapsed_time(e1) * 1e3 / args.iters
                res.setdefault(f"v{v}_mb{mb:g}", []).append(round(us, 2))
                print(f"variant {v} rot {mb:g} MB: {us:.2f} us/iteration", flush=True)
    H = plan.H64.cpu().numpy()
    print(json.dumps({"lib": os.environ.get("CNMF_HIP_LIB", "default"), "us_per_iteration": res,
                      "H_finite": bool(np.isfinite(H).all())}), flush=True)


if __name__ == "__main__":
    main()
