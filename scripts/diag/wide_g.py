"""Diagnostic: where does the forward of the wide_g fixture differ from the golden output?"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgp-rf-mcmc_amd"), os.path.join(ROOT, "tests")]
import test_gpu_parity as T  # noqa: E402

g = dict(np.load(os.path.join(ROOT, "tests/golden/wide_g.npz")))
m = T.model_from_fixture(g)
L = m.n_hidden_layers
F = T.cpu(m.BNN(g["X"]))
ref = g[f"F{L - 1}"]
err = np.abs(F - ref) / (np.abs(ref).max() + 1e-30)
bad = np.argwhere(err > 1e-4)
print("shape", F.shape, "bad", len(bad))
rows = sorted(set(bad[:, 0].tolist()))
cols = sorted(set(bad[:, 1].tolist()))
print("bad rows", rows[:40], "... n", len(rows))
print("bad cols", cols)
