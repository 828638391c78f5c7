"""Full-Bayes step profiling driver (config 2): run_sgmcmc(full_bayesian=True) for --steps steps,
plus a host-side timing of PredictiveLSE.add_sample (Python overhead per predictive sample).
Run under `rocprofv3 --kernel-trace --stats -- python3 scripts/prof_fb.py`."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dgp-rf-mcmc_amd"))
import torch  # noqa: E402

from dgprf import engine as E  # noqa: E402
from dgprf.data import regression_data  # noqa: E402
from dgprf.predictive import PredictiveLSE  # noqa: E402
from likelihoods import Gaussian  # noqa: E402
from models.regression_model import RegressionDGP  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=1000)
ap.add_argument("--host-reps", type=int, default=200)
args = ap.parse_args()
dev = torch.device("cuda", 0)
N_, B = 1_000_000, 200
X, Y, a = regression_data(N_, 8, seed=0, device=dev)
E.set_seed(7)
m = RegressionDGP(8, 1, n_hidden_layers=3, n_rf=1024, n_gp=[8, 8, 1],
                  likelihood=Gaussian(variance=0.1))
m.precond_update(None, N_, precond_type="identity", full_bayesian=True)
run = dict(batch_size=B, lr=0.01, momentum_decay=0.9, temperature=1.0, steps_per_graph=100)
m.run_sgmcmc(X, Y, N_, 100, full_bayesian=True, **run)
torch.cuda.synchronize()
t0 = time.perf_counter()
m.run_sgmcmc(X, Y, N_, args.steps, full_bayesian=True, **run)
torch.cuda.synchronize()
print(f"full-Bayes: {(time.perf_counter() - t0) * 1e6 / args.steps:.2f} us/step")
m.run_sgmcmc(X, Y, N_, args.steps, **run)
torch.cuda.synchronize()
t0 = time.perf_counter()
m.run_sgmcmc(X, Y, N_, args.steps, **run)
torch.cuda.synchronize()
print(f"W-only: {(time.perf_counter() - t0) * 1e6 / args.steps:.2f} us/step")
# host cost of one predictive add_sample call (tiny test set: the kernel is negligible)
Xt, Yt, _ = regression_data(256, 8, seed=1, device=dev, a=a)
acc = PredictiveLSE(m._engine, Xt, Yt)
acc.add_sample()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(args.host_reps):
    acc.add_sample(build=False)
t_host = (time.perf_counter() - t0) / args.host_reps
torch.cuda.synchronize()
print(f"add_sample host: {t_host * 1e6:.1f} us/call")
