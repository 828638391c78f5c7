"""Profiling driver: predictive forward of the config-2 model on the 1e5-row test set.

  rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pred -o run --output-format csv -- \
      python3 scripts/prof_predict.py --samples 20
  rocprofv3 --pmc SQ_WAVE_CYCLES ... --output-format csv -d ... -- python3 scripts/prof_predict.py
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgp-rf-mcmc_amd")]

from dgprf import engine as E  # noqa: E402
from dgprf.data import regression_data  # noqa: E402
from dgprf.predictive import PredictiveLSE  # noqa: E402
from likelihoods import Gaussian  # noqa: E402
from models.regression_model import RegressionDGP  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--samples", type=int, default=10)
ap.add_argument("--n-test", type=int, default=100_000)
ap.add_argument("--pairs", action="store_true", help="two samples per pass (add_samples)")
ap.add_argument("--batch", action="store_true",
                help="all --samples samples in ONE add_samples call (every pair in one launch)")
args = ap.parse_args()
dev = torch.device("cuda", 0)
_, _, a = regression_data(1000, 8, seed=0, device=dev)
Xt, Yt, _ = regression_data(args.n_test, 8, seed=1, device=dev, a=a)
E.set_seed(2)
m = RegressionDGP(8, 1, n_hidden_layers=3, n_rf=1024, n_gp=[8, 8, 1], likelihood=Gaussian(variance=0.1))
m.precond_update(None, 1_000_000, precond_type="identity")
acc = PredictiveLSE(m._engine, Xt, Yt)
th = torch.stack([m._engine.theta.clone(), m._engine.theta.clone()])
if args.pairs:
    th[1].mul_(0.5)
    acc.add_samples(th)
else:
    acc.add_sample()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
if args.batch:
    thb = torch.stack([m._engine.theta.clone() * (1.0 - 0.01 * i) for i in range(args.samples)])
    acc.add_samples(thb, build=False)  # scratch allocation and first launch outside the clock
    torch.cuda.synchronize()
    ev0.record()
    acc.add_samples(thb, build=False)
    ev1.record()
    torch.cuda.synchronize()
    print(f"predictive (batch of {args.samples}): {ev0.elapsed_time(ev1) / args.samples * 1e3:.1f} "
          f"us/sample; finalize {acc.finalize()}")
    sys.exit(0)
ev0.record()
for _ in range(args.samples // (2 if args.pairs else 1)):
    if args.pairs:
        acc.add_samples(th, build=False)
    else:
        acc.add_sample(build=False)
ev1.record()
torch.cuda.synchronize()
k = args.samples // (2 if args.pairs else 1) * (2 if args.pairs else 1)
print(f"predictive{' (pairs)' if args.pairs else ''}: {ev0.elapsed_time(ev1) / k * 1e3:.1f} us/sample; "
      f"finalize {acc.finalize()}")  # (the same numbers for every library build: a parity check)
