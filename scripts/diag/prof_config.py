"""Diagnostic: per-kernel event times of one SGHMC step for a BASELINE config (default 4), and the
predictive us/sample over the config's test-set size (capped at 100k rows)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgp-rf-mcmc_amd")]
from dgprf import engine as E  # noqa: E402
from dgprf.data import CONFIGS, classification_data, regression_data  # noqa: E402
from likelihoods import Gaussian, Softmax  # noqa: E402
from models.dgp import DGP_RF  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 4
c = CONFIGS[cfg]
dev = torch.device("cuda", 0)
if c["likelihood"] == "softmax":
    X, Y = classification_data(c["n"], c["d_in"], c["d_out"], seed=0, device=dev)
    lik = Softmax()
else:
    X, Y, _ = regression_data(c["n"], c["d_in"], seed=0, device=dev)
    lik = Gaussian(variance=c["variance"])
E.set_seed(3)
m = DGP_RF(c["d_in"], c["d_out"], n_hidden_layers=len(c["kinds"]), n_rf=c["n_rf"],
           n_gp=c["n_gp"], likelihood=lik, kernel_type_list=c["kinds"])
m.precond_update(None, c["n"], precond_type="identity")
prof = m._engine.profile_step(X, Y, c["batch"], c["n"], 0.01, 0.9, 1.0, reps=100)
e = prof["empty"]
print(f"config {cfg}: empty pair {e * 1e3:.2f} us")
print("fwd  us:", [round((x - e) * 1e3, 2) for x in prof["fwd"]])
print("bwd  us:", [round((x - e) * 1e3, 2) for x in prof["bwd"]])
print("upd  us:", round((prof["update"] - e) * 1e3, 2))

from dgprf.predictive import PredictiveLSE  # noqa: E402
nt = min(c["n_test"], 100_000)
if c["likelihood"] == "softmax":
    Xt, Yt = classification_data(nt, c["d_in"], c["d_out"], seed=1, device=dev)
else:
    Xt, Yt, _ = regression_data(nt, c["d_in"], seed=1, device=dev)
acc = PredictiveLSE(m._engine, Xt, Yt)
acc.add_sample()
acc.add_sample()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    acc.add_sample(build=False)
e1.record()
torch.cuda.synchronize()
print(f"predictive us/sample (n_test={nt}): {e0.elapsed_time(e1) / 10 * 1e3:.1f}")
