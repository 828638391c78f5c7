"""Diagnostic: the driver's short bench shape (--steps 20 --warmup 5) on config 2 — wall time of
one timed run_sgmcmc call (bench.py's timed region: barrier/sync, replays, sync) for several
steps_per_graph values, with the host-side pieces timed on their own."""
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

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
spgs = [int(s) for s in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 2, 4, 5, 10, 20]
trials = 15
dev = torch.device("cuda", 0)
N_, B = 1_000_000, 200
X, Y, _ = regression_data(N_, 8, seed=0, device=dev)
E.set_seed(2)
m = RegressionDGP(8, 1, n_hidden_layers=3, n_rf=[1024] * 3, n_gp=[8, 8, 1],
                  likelihood=Gaussian(variance=0.1))
m.precond_update(None, N_, precond_type="identity")
sync = torch.cuda.synchronize

t = []
for _ in range(50):
    sync()
    t0 = time.perf_counter()
    sync()
    t.append(time.perf_counter() - t0)
print(f"idle synchronize: {statistics.median(t) * 1e6:.1f} us", flush=True)
t = []
for _ in range(50):
    sync()
    t0 = time.perf_counter()
    m._engine.build_omega()
    sync()
    t.append(time.perf_counter() - t0)
print(f"build_omega + sync: {statistics.median(t) * 1e6:.1f} us", flush=True)

for spg in spgs:
    run = dict(batch_size=B, lr=0.01, momentum_decay=0.9, temperature=1.0, steps_per_graph=spg)
    for g, _ in m.sgmcmc_graphs(X, Y, N_, K, **run):
        g.launch()
    m.run_sgmcmc(X, Y, N_, 5, **run)
    walls, hosts, devs = [], [], []
    for _ in range(trials):
        sync()
        sync()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        m.run_sgmcmc(X, Y, N_, K, **run)
        e1.record()
        t1 = time.perf_counter()
        sync()
        sync()
        t2 = time.perf_counter()
        walls.append(t2 - t0)
        hosts.append(t1 - t0)
        devs.append(e0.elapsed_time(e1) * 1e-3)
    w = statistics.median(walls)
    print(f"  first trials (us/step): {[round(x * 1e6 / K, 2) for x in walls[:3]]}")
    print(f"K={K} spg={spg}: wall {w * 1e6 / K:.2f} us/step ({K / w:.0f} steps/s), host call "
          f"{statistics.median(hosts) * 1e6:.0f} us, events {statistics.median(devs) * 1e6 / K:.2f} "
          f"us/step, min wall {min(walls) * 1e6 / K:.2f}", flush=True)

# head + rest plans: a short first graph reaches the GPU sooner while the host submits the rest
from dgprf import _native as N  # noqa: E402
eng = m._engine
mk = lambda k: eng.graph(X, Y, B, N_, 0.01, 0.9, 1.0, k, N.SCHED_CONST, 0, 1, False, 0)
for plan in ([20], [1, 19], [2, 18], [4, 16], [10, 10]):
    gs = [mk(k) for k in plan]
    for g in gs:
        g.launch()
    walls = []
    for _ in range(trials):
        sync()
        sync()
        t0 = time.perf_counter()
        eng.build_omega()
        for g in gs:
            g.launch()
        sync()
        sync()
        walls.append(time.perf_counter() - t0)
    w = statistics.median(walls)
    print(f"plan {plan}: wall {w * 1e6 / K:.2f} us/step (min {min(walls) * 1e6 / K:.2f}, "
          f"first {walls[0] * 1e6 / K:.2f})", flush=True)
