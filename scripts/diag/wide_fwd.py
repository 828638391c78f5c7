"""Diagnostic: forward of a wide-first-layer model (config-4 shapes) against the oracle for several
row counts, through the tile kernel (default), the row kernel (DGPRF_FORWARD_ROWS) and without the
A_1 GEMM (DGPRF_FORWARD_NO_AGEMM) — set by the caller's environment."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgp-rf-mcmc_amd")]
from oracle import dgp_oracle as O  # noqa: E402
from dgprf import engine as E  # noqa: E402
from likelihoods import Softmax  # noqa: E402
from models.dgp import DGP_RF  # noqa: E402


def cpu(t):
    return t.detach().double().cpu().numpy()


E.set_seed(14)
kinds, n_rf, n_gp, D = ["RBF"] * 4, [4096] * 4, [30, 30, 30, 10], 784
m = DGP_RF(D, 10, n_hidden_layers=4, n_rf=n_rf, n_gp=n_gp, likelihood=Softmax(), kernel_type_list=kinds)
p = O.Params(D, 10, n_rf, n_gp, kinds, "softmax", False,
             z=[cpu(m.BNN.layers[2 * l].z) for l in range(4)], W=[cpu(w) for w in m.W_mcmc],
             log_inv_ls=[cpu(k.log_inv_length_scale) for k in m.kernel_list])
rng = np.random.default_rng(0)
for n in (32, 64, 100, 1000):
    X = rng.uniform(-0.5, 0.5, (n, D)).astype(np.float32).astype(np.float64)
    outs = m._engine.forward(X, f_out="all")["F"]
    _, cache = O.forward(p, X, keep=True)
    errs = []
    for l in range(4):
        Fo = cache[l][2] @ p.W[l]
        F = cpu(outs[l][0])
        errs.append(float(np.max(np.abs(F - Fo)) / np.max(np.abs(Fo))))
    print(n, ["%.1e" % e for e in errs], flush=True)
