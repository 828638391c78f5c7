"""Diagnostic: predictive add_samples time of BASELINE config 3/4/5 (bench_config's predictive leg
without the steps), for A/B of variant libraries (DGPRF_LIB).  Prints us per sample and a checksum
of the accumulators so two builds can be compared for identical bits.

  python scripts/diag/pred_config.py 4 [samples] [reps]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgp-rf-mcmc_amd")]
from dgprf import engine as E  # noqa: E402
from dgprf.data import CONFIGS, classification_data, regression_data  # noqa: E402
from dgprf.predictive import PredictiveLSE  # noqa: E402
from likelihoods import Gaussian, Softmax  # noqa: E402
from models.dgp import DGP_RF  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 4
S = int(sys.argv[2]) if len(sys.argv) > 2 else 10
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
dev = torch.device("cuda", 0)
c = CONFIGS[cfg]
n, nt = c["n"], c["n_test"]
if c["likelihood"] == "softmax":
    X, Y = classification_data(n, c["d_in"], c["d_out"], seed=0, device=dev)
    Xt, Yt = classification_data(nt, c["d_in"], c["d_out"], seed=1, device=dev)
    lik = Softmax()
else:
    X, Y, a = regression_data(n, c["d_in"], seed=0, device=dev)
    Xt, Yt, _ = regression_data(nt, c["d_in"], seed=1, device=dev, a=a)
    lik = Gaussian(variance=c["variance"])
E.set_seed(20 + cfg)
m = DGP_RF(c["d_in"], c["d_out"], n_hidden_layers=len(c["kinds"]), n_rf=c["n_rf"], n_gp=c["n_gp"],
           likelihood=lik, kernel_type_list=c["kinds"])
m.precond_update(None, n, precond_type="identity")
run = dict(batch_size=c["batch"], lr=c["lr"], momentum_decay=c["beta"], temperature=c["T"],
           steps_per_graph=100, perm_seed=cfg)
m.run_sgmcmc(X, Y, n, 100, **run)
th = []
for _ in range(S):
    m.run_sgmcmc(X, Y, n, 1, **run)
    th.append(m._engine.theta.clone())
th = torch.stack(th)
acc = PredictiveLSE(m._engine, Xt, Yt)
acc.add_samples(th)
torch.cuda.synchronize()
ts = []
for _ in range(reps):
    acc = PredictiveLSE(m._engine, Xt, Yt)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    acc.add_samples(th, build=False)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) * 1e3 / S)
ck = float(acc.m.double().sum() + acc.s.double().sum() + (acc.e.double().sum() if acc.e is not None else 0))
print(f"config {cfg} S {S}: us/sample min {min(ts):.1f} median {sorted(ts)[len(ts) // 2]:.1f}  "
      f"checksum {ck!r}", flush=True)
