"""Diagnostic: per-layer gradient error of the large-batch backward against the oracle for a few
shapes (run with and without DGPRF_NO_RW=1 to compare the row-wave and row-group kernels)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgp-rf-mcmc_amd"), os.path.join(ROOT, "tests")]
from oracle import dgp_oracle as O  # noqa: E402
from test_gpu_large_batch import _model, _oracle  # noqa: E402
from test_gpu_parity import rel_err, unpack  # noqa: E402

SHAPES = [
    (["ARC"] * 3, [1024] * 3, [8, 8, 1], 8, False, "gaussian", 2048),
    (["ARC"] * 3, [2048] * 3, [8, 8, 1], 8, False, "gaussian", 4096),
    (["ARC"] * 3, [2048] * 3, [4, 4, 1], 4, False, "gaussian", 2048),
    (["ARC"] * 3, [2048] * 3, [9, 9, 1], 9, False, "gaussian", 2048),
    (["ARC"] * 3, [1024] * 3, [9, 9, 1], 9, False, "gaussian", 2048),
    (["ARC"] * 3, [2048] * 3, [8, 8, 1], 8, False, "gaussian", 2048),
    (["RBF"] * 3, [1024] * 3, [9, 9, 1], 9, False, "gaussian", 2048),
    (["RBF"] * 3, [1024] * 3, [8, 8, 1], 8, False, "gaussian", 2048),
]
for i, (kinds, n_rf, n_gp, d_in, cat, lik, B) in enumerate(SHAPES):
    m = _model(kinds, n_rf, n_gp, d_in, cat, lik, 70 + i)
    p = _oracle(m, kinds, n_rf, n_gp, d_in, cat, lik)
    rng = np.random.default_rng(i)
    X = rng.standard_normal((B, d_in))
    Y = rng.standard_normal((B, n_gp[-1]))
    G = unpack(m._engine, m._engine.grad(X, Y, 50_000))
    ref = O.grad_W(p, X, Y, 50_000)
    print(i, kinds[0], n_rf[0], n_gp, "errs", [f"{rel_err(G[l], ref[l]):.2e}" for l in range(3)], flush=True)
