"""A/B of the folded update (plan.ipu) against the separate update kernel (Engine.set_separate_update)
on graph-replayed SGHMC steps of BASELINE configs at B = 200, interleaved over rounds.

  python scripts/diag/ipu_ab.py [configs, e.g. 2,3] [steps] [rounds]
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

cfgs = [int(c) for c in sys.argv[1].split(",")] if len(sys.argv) > 1 else [2, 3]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
dev = torch.device("cuda", 0)
for cfg in cfgs:
    c = CONFIGS[cfg]
    if c["likelihood"] == "softmax":
        X, Y = classification_data(c["n"], c["d_in"], c["d_out"], seed=0, device=dev)
        lik = Softmax()
    else:
        X, Y, _ = regression_data(c["n"], c["d_in"], seed=0, device=dev)
        lik = Gaussian(variance=c["variance"])
    models = {}
    for name, sep in (("folded", False), ("separate", True)):
        E.set_seed(3)
        m = DGP_RF(c["d_in"], c["d_out"], n_hidden_layers=len(c["kinds"]), n_rf=c["n_rf"],
                   n_gp=c["n_gp"], likelihood=lik, kernel_type_list=c["kinds"])
        m.precond_update(None, c["n"], precond_type="identity")
        m._engine.set_separate_update(sep)
        models[name] = m
    run = dict(batch_size=c["batch"], lr=c["lr"], momentum_decay=c["beta"], temperature=c["T"],
               steps_per_graph=100)
    for m in models.values():
        m.run_sgmcmc(X, Y, c["n"], 200, **run)
    torch.cuda.synchronize()
    res = {k: [] for k in models}
    for _ in range(rounds):
        for name, m in models.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            m.run_sgmcmc(X, Y, c["n"], steps, **run)
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) * 1e3 / steps)
    ipu = models["folded"]._engine.plan_ws(c["batch"])[0].ipu
    print(f"config {cfg} (plan.ipu={ipu}): " + "; ".join(
        f"{k} {' / '.join(f'{v:.2f}' for v in vs)} us/step" for k, vs in res.items()), flush=True)
    del models
    torch.cuda.empty_cache()
