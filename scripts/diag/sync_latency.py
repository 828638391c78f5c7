"""Diagnostic: host-side latency around a timed 20-step graph replay (the driver's bench shape):
wall time with torch.cuda.synchronize() alone vs polling the closing event first (then the same
synchronize), and after an idle gap of 1 / 10 / 100 ms, against the events' device span."""
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgp-rf-mcmc_amd")]
from dgprf import engine as E  # noqa: E402
from dgprf.data import regression_data  # noqa: E402
from likelihoods import Gaussian  # noqa: E402
from models.regression_model import RegressionDGP  # noqa: E402

K = 20
dev = torch.device("cuda", 0)
X, Y, _ = regression_data(1_000_000, 8, seed=0, device=dev)
E.set_seed(2)
m = RegressionDGP(8, 1, n_hidden_layers=3, n_rf=[1024] * 3, n_gp=[8, 8, 1],
                  likelihood=Gaussian(variance=0.1))
m.precond_update(None, 1_000_000, precond_type="identity")
run = dict(batch_size=200, lr=0.01, momentum_decay=0.9, temperature=1.0, steps_per_graph=100)
plan = m.sgmcmc_graphs(X, Y, 1_000_000, K, **run)
for g, _ in plan:
    g.launch()
torch.cuda.synchronize()
for mode in ("sync", "poll", "idle1ms", "idle10ms", "idle100ms", "sync"):
    walls, devs = [], []
    for _ in range(15):
        torch.cuda.synchronize()
        if mode.startswith("idle"):  # host-side idle gap before the timed replay
            time.sleep(float(mode[4:-2]) * 1e-3)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        for g, reps in plan:
            for _ in range(reps):
                g.launch()
        e1.record()
        if mode == "poll":
            while not e1.query():
                pass
        torch.cuda.synchronize()
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t0)
        devs.append(e0.elapsed_time(e1) * 1e-3)
    print(f"{mode}: wall {statistics.median(walls) * 1e6 / K:.2f} us/step, events "
          f"{statistics.median(devs) * 1e6 / K:.2f} us/step, first {walls[0] * 1e6 / K:.2f}", flush=True)
