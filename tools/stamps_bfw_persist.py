"""End-of-iteration phases of the persistent cfg4 launch (mu_iter_bfw_kernel) from the stamps build:
thread 0 of every workgroup sums s_memtime deltas per phase; printed as cycles per (workgroup,
iteration) and µs at the clock the launch ran (cycles / wall of the same launch).

    python -m cnmf_amd.build --stamps
    CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_stamps.so python tools/stamps_bfw_persist.py
"""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
NAMES = ["", "waves' sums -> partial row (stores issued)", "barrier A", "reduce-scatter", "barrier B",
         "AB -> LDS", "basis update + HHt (f64 MFMA)", "H terms + pads", "partial row stores retired"]


def main():
    import torch
    from cnmf_amd import _lib
    from cnmf_amd.solver import MUPlan
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(1_000_000, 300, seed=0, dtype=np.float32)
    W0, H0 = random_init(X, 16, 42)
    lib = _lib.load()
    fn = lib.cnmf_debug_eoi
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    fn.restype = ctypes.c_int
    plan = MUPlan(torch.from_numpy(X).cuda().to(torch.bfloat16), 16)
    plan.set_W(torch.from_numpy(W0))
    plan.set_H(torch.from_numpy(H0))
    print(plan.describe(), flush=True)
    plan.iterate(20)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 16)()
    fn(buf, 1)
    n = 50
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    plan.iterate(n)
    e1.record()
    torch.cuda.synchronize()
    plan.check_sync_error()
    us = e0.elapsed_time(e1) * 1e3 / n
    fn(buf, 1)
    pairs = max(buf[15], 1)
    out = {"us_per_iteration": round(us, 2), "wg_iterations": int(pairs)}
    for i in range(1, 9):
        out[NAMES[i]] = round(buf[i] / pairs, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
