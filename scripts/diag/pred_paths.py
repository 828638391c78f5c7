"""Diagnostic: predictive us/sample of a BASELINE config through each forward path (tile kernel,
row kernel) on the config's test-set size (capped at 100k rows)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgp-rf-mcmc_amd")]
from dgprf import _native as N  # noqa: E402
from dgprf import engine as E  # noqa: E402
from dgprf.data import CONFIGS, classification_data, regression_data  # noqa: E402
from dgprf.predictive import PredictiveLSE  # noqa: E402
from likelihoods import Gaussian, Softmax  # noqa: E402
from models.dgp import DGP_RF  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
paths = sys.argv[2].split(",") if len(sys.argv) > 2 else ["auto", "rows"]
nt = int(sys.argv[3]) if len(sys.argv) > 3 else None
c = CONFIGS[cfg]
dev = torch.device("cuda", 0)
nt = nt or min(c["n_test"], 100_000)
if c["likelihood"] == "softmax":
    Xt, Yt = classification_data(nt, c["d_in"], c["d_out"], seed=1, device=dev)
    lik = Softmax()
else:
    Xt, Yt, _ = regression_data(nt, c["d_in"], seed=1, device=dev)
    lik = Gaussian(variance=c["variance"])
E.set_seed(3)
m = DGP_RF(c["d_in"], c["d_out"], n_hidden_layers=len(c["kinds"]), n_rf=c["n_rf"],
           n_gp=c["n_gp"], likelihood=lik, kernel_type_list=c["kinds"])
code = {"auto": N.FWD_AUTO, "rows": N.FWD_ROWS, "noagemm": N.FWD_NO_AGEMM, "tile": N.FWD_TILE,
        "rows16": N.FWD_ROWS16, "rows8": N.FWD_ROWS8}
pl = m._engine.layout
flops = nt * sum(2 * (pl.d[l] * pl.n_rf[l] + pl.P[l] * pl.n_gp[l]) for l in range(pl.n_layers))
for p in paths:
    m._engine.set_forward_path(code[p])
    acc = PredictiveLSE(m._engine, Xt, Yt)
    acc.add_sample()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    S = 20
    e0.record()
    t0 = time.perf_counter()
    for _ in range(S):
        acc.add_sample(build=False)
    host_us = (time.perf_counter() - t0) * 1e6 / S
    e1.record()
    torch.cuda.synchronize()
    print(f"  host enqueue {host_us:.1f} us/sample", flush=True)
    us = e0.elapsed_time(e1) * 1e3 / S
    print(f"config {cfg} N_t={nt} path={p}: {us:.1f} us/sample, "
          f"{flops / us / 1e6:.1f} TFLOP/s = {flops / us / 1e6 / 157.3 * 100:.1f} % of fp32 MFMA peak",
          flush=True)
