"""Diagnostic: per-layer relative error of the device W gradient and per-layer forward outputs
against the float64 oracle for deep / wide configurations (config-5 family)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgp-rf-mcmc_amd"), os.path.join(ROOT, "tests")]
from oracle import dgp_oracle as O  # noqa: E402
from dgprf import engine as E  # noqa: E402
from likelihoods import Gaussian  # noqa: E402
from models.dgp import DGP_RF  # noqa: E402


def cpu(t):
    return t.detach().double().cpu().numpy()


def rel(a, b):
    return float(np.max(np.abs(a - b)) / (np.max(np.abs(b)) + 1e-30))


def run(name, kinds, n_rf, n_gp, D, B=48, seed=7, xseed=3):
    E.set_seed(seed)
    m = DGP_RF(D, n_gp[-1], n_hidden_layers=len(kinds), n_rf=n_rf, n_gp=n_gp,
               likelihood=Gaussian(variance=0.1), kernel_type_list=kinds)
    p = O.Params(D, n_gp[-1], n_rf, n_gp, kinds, "gaussian", False,
                 z=[cpu(m.BNN.layers[2 * l].z) for l in range(len(kinds))],
                 W=[cpu(w) for w in m.W_mcmc],
                 log_inv_ls=[cpu(k.log_inv_length_scale) for k in m.kernel_list],
                 lik_log_var=np.log(0.1))
    rng = np.random.default_rng(xseed)
    X = rng.standard_normal((B, D)).astype(np.float32).astype(np.float64)
    Y = rng.standard_normal((B, n_gp[-1])).astype(np.float32).astype(np.float64)
    eng = m._engine
    Fs = eng.forward(X, f_out="all")["F"]
    _, cache = O.forward(p, X, keep=True)
    ferr = []
    Fo = X
    for l in range(len(kinds)):
        Fo = cache[l][2] @ p.W[l]
        ferr.append(rel(cpu(Fs[l][0]), Fo))
    G = eng.grad(X, Y, 1e7)
    ref = O.grad_W(p, X, Y, 1e7)
    pl = eng.layout
    gerr = []
    for l in range(len(kinds)):
        o, P, g = pl.w_off[l], pl.P[l], pl.n_gp[l]
        gerr.append(rel(cpu(G[0, o:o + P * g]).reshape(P, g), ref[l]))
    amax = [float(np.max(np.abs(cache[l][1]))) for l in range(len(kinds))]
    near = [int(np.sum(np.abs(cache[l][1]) < 1e-5)) if kinds[l] == "ARC" else 0
            for l in range(len(kinds))]
    p32 = O.Params(D, n_gp[-1], n_rf, n_gp, kinds, "gaussian", False, z=p.z, W=p.W,
                   log_inv_ls=p.log_inv_ls, lik_log_var=np.log(0.1), dtype=np.float32)
    r32 = O.grad_W(p32, X.astype(np.float32), Y.astype(np.float32), 1e7)
    e32 = [rel(r32[l].astype(np.float64), ref[l]) for l in range(len(kinds))]
    print(f"{name:28s} |A|<1e-5 in ARC layers {near}  fp32-oracle gW err {['%.1e' % e for e in e32]}")
    print(f"{name:28s} F err {['%.1e' % e for e in ferr]}  gW err {['%.1e' % e for e in gerr]}  "
          f"max|A| {['%.0f' % a for a in amax]}", flush=True)


run("config5 test seed", ["RBF", "ARC", "RBF", "ARC", "RBF"], [8192] * 5, [16, 16, 16, 16, 1], 16,
    seed=15, xseed=5)
run("config5", ["RBF", "ARC", "RBF", "ARC", "RBF"], [8192] * 5, [16, 16, 16, 16, 1], 16)
