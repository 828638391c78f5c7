"""Diagnostic: graph-replayed SGHMC steps of config 2 (or another BASELINE config) at one or more
minibatch sizes, timed with events over K replayed steps; run under
`rocprofv3 --kernel-trace --stats` for per-kernel durations.

  python scripts/diag/step_graph.py [config] [B1,B2,...] [steps]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgp-rf-mcmc_amd")]
from dgprf import engine as E  # noqa: E402
from dgprf.data import CONFIGS, classification_data, regression_data  # noqa: E402
from likelihoods import Gaussian, Softmax  # noqa: E402
from models.dgp import DGP_RF  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
c = CONFIGS[cfg]
batches = [int(b) for b in sys.argv[2].split(",")] if len(sys.argv) > 2 else [c["batch"]]
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 2000
dev = torch.device("cuda", 0)
if c["likelihood"] == "softmax":
    X, Y = classification_data(c["n"], c["d_in"], c["d_out"], seed=0, device=dev)
    lik = Softmax()
else:
    X, Y, _ = regression_data(c["n"], c["d_in"], seed=0, device=dev)
    lik = Gaussian(variance=c["variance"])
for B in batches:
    E.set_seed(3)
    m = DGP_RF(c["d_in"], c["d_out"], n_hidden_layers=len(c["kinds"]), n_rf=c["n_rf"],
               n_gp=c["n_gp"], likelihood=lik, kernel_type_list=c["kinds"])
    m.precond_update(None, c["n"], precond_type="identity")
    if os.environ.get("DGPRF_DIAG_NO_A1"):  # per-step A_1 GEMM instead of the resident projection
        m._engine.resident_a1 = False
    if os.environ.get("DGPRF_DIAG_FWD"):  # forward path of the fused step forward (diagnostic)
        from dgprf import _native as N
        m._engine.set_forward_path(getattr(N, "FWD_" + os.environ["DGPRF_DIAG_FWD"].upper()))
    spg = 100 if B <= 1024 else 10
    run = dict(batch_size=B, lr=c["lr"], momentum_decay=c["beta"], temperature=c["T"],
               steps_per_graph=spg)
    k = max(spg, steps // spg * spg) if B <= 1024 else max(spg, steps // 10 // spg * spg)
    m.run_sgmcmc(X, Y, c["n"], 2 * spg, **run)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    m.run_sgmcmc(X, Y, c["n"], k, **run)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / k
    pl = m._engine.plan_ws(B)[0]
    print(f"config {cfg} B={B}: {us:.2f} us/step ({1e6 / us:.0f} steps/s), ws {pl.ws_chain * 4 / 1e6:.1f} MB",
          flush=True)
    del m
