"""Per-phase cycle breakdown of the bf16 MFMA pass (cfg4: 1e6 x 300 bf16, k = 16) from the stamps build.

    python -m cnmf_amd.build --stamps
    CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_stamps.so python tools/stamps_bf16.py
"""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
NAMES = ["", "stage wait+LDS write", "staging barrier", "prefetch issue", "phase 1", "phase 2 + barrier",
         "phase 3 + end barrier"]
# mu_pass_bfw_kernel (wave tiles, a pair per body; cycles per wave tile of 16 samples)
NAMES_BFW = ["", "waits + staging", "prefetch issue", "phase 1 (the pair)", "phases 2+3, first tile",
             "phases 2+3, second tile", "-"]


def main():
    import torch
    from cnmf_amd import _lib
    from cnmf_amd.solver import MUPlan
    from cnmf_amd.synthetic import iop_spectra, random_init
    k = int(os.environ.get("K", "16"))
    X = iop_spectra(1_000_000, 300, seed=0, dtype=np.float32)
    W0, H0 = random_init(X, k, 42)
    lib = _lib.load()
    fn = lib.cnmf_debug_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    fn.restype = ctypes.c_int
    plan = MUPlan(torch.from_numpy(X).cuda().to(torch.bfloat16), k)
    plan.set_W(torch.from_numpy(W0))
    plan.set_H(torch.from_numpy(H0))
    plan.iterate(3)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 16)()
    fn(buf, 1)
    n = 20
    for flags in (3, 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            plan.sample_pass(flags)
        e1.record()
        torch.cuda.synchronize()
        pass_us = e0.elapsed_time(e1) * 1e3 / n
        fn(buf, 1)
        waves = buf[8]
        tiles_per_wave = (plan.n_rows / 64) / plan.n_parts
        out = {"flags": flags, "waves": waves, "pass_us": round(pass_us, 2), "tiles_per_wave": round(tiles_per_wave, 2)}
        tot = 0
        names = NAMES_BFW if os.environ.get("BFW", "1") == "1" else NAMES
        for i in range(1, 7):
            cyc = buf[i] / waves / tiles_per_wave
            tot += cyc
            out[names[i]] = round(cyc, 1)
        out["total_cycles_per_tile"] = round(tot, 1)
        out["implied_GHz"] = round(tot * tiles_per_wave / (pass_us * 1e3), 3)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
