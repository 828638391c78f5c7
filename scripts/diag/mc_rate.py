"""Diagnostic: aggregate chain-steps/s of C chains per GPU (config 2, B = 200, graph of 50 steps),
for each C on the command line — bench.py's multi_chain leg at several chain counts.

  python scripts/diag/mc_rate.py 2,4,8,16,64
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgp-rf-mcmc_amd")]
from dgprf import _native as N  # noqa: E402
from dgprf import engine as E  # noqa: E402
from dgprf.data import regression_data  # noqa: E402

Cs = [int(c) for c in (sys.argv[1] if len(sys.argv) > 1 else "2,4,8,16,64").split(",")]
dev = torch.device("cuda", 0)
X, Y, _ = regression_data(1_000_000, 8, seed=0, device=dev)
spec = E.ModelSpec(8, 1, [N.RBF] * 3, [1024] * 3, [8, 8, 1])
out = []
for C in Cs:
    e = E.Engine(spec, C, seed=5)
    E.normal(None, N.RNG_Z, out=e.z)
    E.normal(None, N.RNG_W, out=e.theta)
    e.init_moments()
    e.build_omega()
    g = e.graph(X, Y, 200, 1_000_000, 0.01, 0.9, 1.0, 50)
    g.launch()
    torch.cuda.synchronize()
    reps = max(4, 400 // C)
    t0 = time.perf_counter()
    for _ in range(reps):
        g.launch()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert torch.isfinite(e.theta).all()
    out.append(f"C={C} ns={list(e.layout.ns[:3])}: {C * reps * 50 / dt:,.0f} chain-steps/s "
               f"({dt * 1e6 / (reps * 50):.1f} us/step)")
    del g, e
print(" | ".join(out), flush=True)
