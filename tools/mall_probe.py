"""Diagnostic: does the Infinity Cache serve re-reads?  (1) back-to-back read sweeps (cnmf_hbm_probe)
over buffers of 64 MB .. 1 GB: GB/s per size; (2) µs per persistent MU iteration (fixed order) at
0.25 .. 2 M rows (cfg2 shape otherwise)."""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from cnmf_amd import _lib
    from cnmf_amd.solver import MUPlan
    from cnmf_amd.synthetic import iop_spectra, random_init
    lib = _lib.load()
    st = torch.cuda.current_stream()
    out = torch.zeros(4096, dtype=torch.float64, device="cuda")
    big = torch.empty(1 << 30, dtype=torch.uint8, device="cuda").fill_(1)
    res = {"sweep_GBps": {}, "mu_us_per_iteration": {}}
    for mb in (64, 128, 192, 240, 256, 288, 324, 400, 512, 1024):
        n = mb << 20
        for _ in range(5):
            lib.cnmf_hbm_probe(big.data_ptr(), n, out.data_ptr(), 2048, st.cuda_stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 30
        e0.record(st)
        for _ in range(reps):
            lib.cnmf_hbm_probe(big.data_ptr(), n, out.data_ptr(), 2048, st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize()
        gbs = n * reps / (e0.elapsed_time(e1) / 1e3) / 1e9
        res["sweep_GBps"][mb] = round(gbs, 1)
        print(f"sweep {mb} MB: {gbs:.1f} GB/s", flush=True)
    del big
    os.environ["CNMF_ROT_MB"] = "0"
    for rows in (250_048, 500_032, 750_016, 1_000_000, 1_500_032, 2_000_000):
        X = iop_spectra(rows, 81, seed=0, dtype=np.float32)
        W0, H0 = random_init(X, 4, 42)
        plan = MUPlan(torch.from_numpy(X).cuda(), 4)
        plan.set_W(torch.from_numpy(W0))
        plan.set_H(torch.from_numpy(H0).cuda())
        plan.iterate(300)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        plan.iterate(300)
        e1.record(st)
        torch.cuda.synchronize()
        plan.check_sync_error()
        us = e0.elapsed_time(e1) * 1e3 / 300
        res["mu_us_per_iteration"][rows] = round(us, 2)
        print(f"MU rows {rows} ({rows * 324 / 1e6:.0f} MB of X): {us:.2f} us/iteration, "
              f"{rows * 324 / us / 1e3:.0f} GB/s of X", flush=True)
        del plan
    print(json.dumps({"lib": os.environ.get("CNMF_HIP_LIB", "default"), **res}), flush=True)


if __name__ == "__main__":
    main()
