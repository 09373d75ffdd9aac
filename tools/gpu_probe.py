"""Step-by-step GPU probe: each C-ABI call followed by a synchronize and an unbuffered print, so a
fault or hang names the call that caused it.  Small shapes only."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def log(msg):
    print(f"[{time.strftime('%H:%M:%S')}] {msg}", flush=True)


def main():
    import torch
    from cnmf_amd import _lib
    from cnmf_amd.solver import MUPlan
    from oracle import mu_ref
    log(f"torch {torch.__version__} device {torch.cuda.get_device_name(0)}")
    lib = _lib.load()
    log(f"lib abi {lib.cnmf_abi_version()}")
    for (N, F, k, dt) in [(100, 81, 4, np.float32), (1037, 81, 5, np.float32), (300, 17, 3, np.float64),
                          (500, 300, 16, np.float32)]:
        rng = np.random.default_rng(0)
        X = rng.random((N, F)).astype(dt)
        W0 = rng.random((N, k)).astype(dt)
        H0 = rng.random((k, F)).astype(dt)
        plan = MUPlan(torch.from_numpy(X).cuda(), k)
        log(f"N={N} F={F} k={k} {dt.__name__}: plan n_parts={plan.n_parts}")
        plan.set_W(torch.from_numpy(W0)); torch.cuda.synchronize(); log("  set_W ok")
        plan.set_H(torch.from_numpy(H0)); torch.cuda.synchronize(); log("  set_H/refresh ok")
        plan.sample_pass(_lib.PASS_UPDATE_W | _lib.PASS_ACCUMULATE); torch.cuda.synchronize(); log("  pass ok")
        plan.reduce(plan.n_out, plan.AB); torch.cuda.synchronize(); log("  reduce ok")
        plan.basis_update(); torch.cuda.synchronize(); log("  basis_update ok")
        e = plan.frobenius_error(); log(f"  loss ok {e:.6g}")
        plan.iterate(3); torch.cuda.synchronize(); log("  iterate(3) ok")
        Wr, Hr, _ = mu_ref.mu_fit(X.astype(np.float64), W0.astype(np.float64), H0.astype(np.float64),
                                  max_iter=4, tol=0)  # 1 manual step + iterate(3)
        W = plan.W.double().cpu().numpy(); H = plan.H64.cpu().numpy()
        log(f"  relW={np.linalg.norm(W-Wr)/np.linalg.norm(Wr):.2e} relH={np.linalg.norm(H-Hr)/np.linalg.norm(Hr):.2e}")
    log("probe done")


if __name__ == "__main__":
    main()
