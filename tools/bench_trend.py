"""Consecutive persistent launches of cfg2 (500 iterations each), timed with HIP events, to see
launch-to-launch variance (clocks / thermals) on the box."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from cnmf_amd.solver import MUPlan
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(1_000_000, 81, seed=0, dtype=np.float32)
    W0, H0 = random_init(X, 4, 42)
    plan = MUPlan(torch.from_numpy(X).cuda(), 4)
    plan.set_W(torch.from_numpy(W0))
    plan.set_H(torch.from_numpy(H0))
    plan.iterate(20)
    torch.cuda.synchronize()
    for rep in range(int(os.environ.get("REPS", "10"))):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        plan.iterate(500)
        e1.record()
        torch.cuda.synchronize()
        print(f"launch {rep}: {e0.elapsed_time(e1) / 500 * 1e3:.2f} us/iter", flush=True)
        if os.environ.get("GAP"):
            time.sleep(float(os.environ["GAP"]))


if __name__ == "__main__":
    main()
