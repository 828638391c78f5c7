"""Diagnostic: aggregate chain-steps/s of C chains per GPU (config 2, B = 200, graph of 50 steps),
for each C on the command line — bench.py's multi_chain leg at several chain counts.

  python scripts/diag/mc_rate.py 2,4,8,16,64 [config]
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgp-rf-mcmc_amd")]
from dgprf import _native as N  # noqa: E402
from dgprf import engine as E  # noqa: E402
from dgprf.data import CONFIGS, classification_data, regression_data  # noqa: E402

Cs = [int(c) for c in (sys.argv[1] if len(sys.argv) > 1 else "2,4,8,16,64").split(",")]
cfg = int(sys.argv[2]) if len(sys.argv) > 2 else 2
dev = torch.device("cuda", 0)
c = CONFIGS[cfg]
n_data = min(c["n"], 1_000_000)
if c["likelihood"] == "softmax":
    X, Y = classification_data(n_data, c["d_in"], c["d_out"], seed=0, device=dev)
else:
    X, Y, _ = regression_data(n_data, c["d_in"], seed=0, device=dev)
spec = E.ModelSpec(c["d_in"], c["d_out"], [N.RBF if k == "RBF" else N.ARC for k in c["kinds"]],
                   c["n_rf"], c["n_gp"],
                   likelihood=N.LIK_SOFTMAX if c["likelihood"] == "softmax" else N.LIK_GAUSSIAN)
out = []
for C in Cs:
    e = E.Engine(spec, C, seed=5)
    E.normal(None, N.RNG_Z, out=e.z)
    E.normal(None, N.RNG_W, out=e.theta)
    e.init_moments()
    e.build_omega()
    g = e.graph(X, Y, 200, n_data, 1e-4, 0.9, 1.0, 50)  # timing: a small step keeps the chains finite
    g.launch()
    torch.cuda.synchronize()
    reps = max(2, (400 if cfg <= 3 else 40) // C)
    t0 = time.perf_counter()
    for _ in range(reps):
        g.launch()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    fin = bool(torch.isfinite(e.theta).all())
    out.append(f"C={C} ns={list(e.layout.ns[:3])}: {C * reps * 50 / dt:,.0f} chain-steps/s "
               f"({dt * 1e6 / (reps * 50):.1f} us/step{'' if fin else ', diverged'})")
    del g, e
print(" | ".join(out), flush=True)
