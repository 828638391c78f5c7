"""Diagnostic: predictive microseconds per sample of BASELINE config 3 / 4 / 5 for each forward path
(N.FWD_*), S samples scored by one PredictiveLSE.add_samples call — the bench's predictive leg.

  python scripts/diag/pred_paths.py [config] [S]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgp-rf-mcmc_amd")]
from dgprf import _native as N  # noqa: E402
from dgprf.data import CONFIGS, classification_data, regression_data  # noqa: E402
from dgprf.predictive import PredictiveLSE  # noqa: E402
from likelihoods import Gaussian, Softmax  # noqa: E402
from models.dgp import DGP_RF  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
S = int(sys.argv[2]) if len(sys.argv) > 2 else 60
dev = torch.device("cuda", 0)
c = CONFIGS[cfg]
nt = c["n_test"]
if c["likelihood"] == "softmax":
    Xt, Yt = classification_data(nt, c["d_in"], c["d_out"], seed=1, device=dev)
    lik = Softmax()
else:
    Xt, Yt, _ = regression_data(nt, c["d_in"], seed=1, device=dev)
    lik = Gaussian(variance=c["variance"])
m = DGP_RF(c["d_in"], c["d_out"], n_hidden_layers=len(c["kinds"]), n_rf=c["n_rf"], n_gp=c["n_gp"],
           likelihood=lik, kernel_type_list=c["kinds"])
eng = m._engine
th = eng.theta.clone() + 0.01 * torch.randn(S, *eng.theta.shape, device=dev)
names = ("AUTO", "TILE", "ROWS", "ROWS8", "ROWS16")
for name in names:  # every path warmed up (scratch / projection / clocks) before any timing
    eng.set_forward_path(getattr(N, "FWD_" + name))
    PredictiveLSE(eng, Xt, Yt).add_samples(th)
torch.cuda.synchronize()
reps = max(3, 120 // S)
best = {n: float("inf") for n in names}
for rnd in range(3):  # rotated order, best of 3 rounds
    for name in names[rnd % len(names):] + names[:rnd % len(names)]:
        eng.set_forward_path(getattr(N, "FWD_" + name))
        acc = PredictiveLSE(eng, Xt, Yt)
        acc.add_samples(th, build=False)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            acc.add_samples(th, build=False)
        e1.record()
        torch.cuda.synchronize()
        best[name] = min(best[name], e0.elapsed_time(e1) * 1e3 / (reps * S))
eng.set_forward_path(N.FWD_AUTO)
print(f"config {cfg} N_t={nt} S={S} us/sample: " + " | ".join(f"{n} {best[n]:.1f}" for n in names),
      flush=True)
