"""Per-kernel timing on the box: HBM read ceiling (cnmf_hbm_probe), the fused pass with and without
the accumulation phase, the loss pass, and the reduce+update tail, each timed with HIP events over
many back-to-back launches (cfg2 shape by default)."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps, stream):
    import torch
    fn()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--features", type=int, default=81)
    ap.add_argument("--k", type=int, default=4)
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--dtype", default="f32")
    a = ap.parse_args()
    import torch
    from cnmf_amd import _lib
    from cnmf_amd.solver import MUPlan
    from cnmf_amd.synthetic import iop_spectra, random_init
    lib = _lib.load()
    dt = {"f32": np.float32, "f64": np.float64, "bf16": np.float32}[a.dtype]
    X = iop_spectra(a.rows, a.features, seed=0, dtype=dt)
    W0, H0 = random_init(X, a.k, 42)
    Xt = torch.from_numpy(X)
    if a.dtype == "bf16":
        Xt = Xt.to(torch.bfloat16)
    Xd = Xt.cuda()
    plan = MUPlan(Xd, a.k)
    plan.set_W(torch.from_numpy(W0))
    plan.set_H(torch.from_numpy(H0))
    stream = torch.cuda.current_stream()
    s = stream.cuda_stream
    out = {"shape": [a.rows, a.features, a.k, a.dtype], "n_parts": plan.n_parts}
    sx = Xd.element_size()
    algo = a.rows * (a.features * sx + 2 * a.k * plan.W.element_size())
    # HBM read ceiling on a 1 GiB buffer and on X itself
    big = torch.empty(1 << 28, dtype=torch.float32, device="cuda")
    big.uniform_()
    cks = torch.zeros(4096, dtype=torch.float64, device="cuda")
    for nb in (1024, 2048, 4096):
        us = timed(lambda: _lib.check(lib.cnmf_hbm_probe(big.data_ptr(), big.numel() * 4, cks.data_ptr(), nb, s)), 20, stream)
        out[f"probe_1GiB_{nb}blk_GBs"] = round(big.numel() * 4 / us / 1e3, 1)
    us = timed(lambda: _lib.check(lib.cnmf_hbm_probe(Xd.data_ptr(), Xd.numel() * sx, cks.data_ptr(), 2048, s)), 100, stream)
    out["probe_X_GBs"] = round(Xd.numel() * sx / us / 1e3, 1)
    for name, flags in (("pass_full", 3), ("pass_no_accum", 1), ("pass_loss", 4)):
        us = timed(lambda: plan.sample_pass(flags), a.reps, stream)
        out[name + "_us"] = round(us, 2)
        out[name + "_GBs"] = round(algo / us / 1e3, 1)

    def tail():
        _lib.check(lib.cnmf_reduce_update(plan.partials.data_ptr(), plan.n_parts, plan.stage.data_ptr(),
                                          plan.counter.data_ptr(), plan.AB.data_ptr(), plan.H64.data_ptr(),
                                          plan.Ht.data_ptr(), plan.HHt.data_ptr(), plan.F, plan.k,
                                          0.0, 0.0, plan.stats.data_ptr(), s))
    out["reduce_update_us"] = round(timed(tail, a.reps, stream), 2)
    us = timed(lambda: plan.iterate(1), a.reps, stream)
    out["iteration_us"] = round(us, 2)
    out["it_per_s"] = round(1e6 / us, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
