"""Debug: one TOL launch of 1 iteration — the device's error at init and its W snapshot vs W0."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from cnmf_amd.solver import ALSPlan
from cnmf_amd.synthetic import iop_spectra

rng = np.random.default_rng(12)
X = iop_spectra(2000, 81, seed=12, dtype=np.float32)
H0 = (rng.random((4, 81)) * X.mean() + 1e-3).astype(np.float32)
W0 = rng.random((2000, 4)).astype(np.float32)
p = ALSPlan(torch.from_numpy(X).cuda(), 4, sum_to_one=1.0, smoothness=0.1)
p.set_W(torch.from_numpy(W0))
p.set_H(torch.from_numpy(H0))
print("host e0", p.frobenius_error())
run, finish = p.prepare_device_tol(1, 1e-3)
p._wsnap.fill_(-7.0)
run()
n, errs = finish()
ws = p._wsnap.cpu().numpy()
print("device", n, errs)
bad = np.argwhere(ws != W0)
print("snapshot mismatches", len(bad), bad[:10], ws[bad[:5, 0]] if len(bad) else None, W0[bad[:5, 0]] if len(bad) else None)
Xd, Hd = X.astype(np.float64), H0.astype(np.float64)
R = Xd - ws.astype(np.float64) @ Hd
print("loss with snapshot W", np.sqrt((R ** 2).sum()))
