"""Diagnostic: the C-chain step against the one-chain step for identical chains (config 2 model,
B = 200).  With a build whose multi-chain plans use fewer feature slices (-DDGPRF_MC_SLICES) the
two engines sum the features in a different order: the gradients agree to float tolerance.

  DGPRF_LIB=scripts/variants/mc4/libdgprf.so python scripts/diag/mc_slices_check.py [chains]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgp-rf-mcmc_amd")]
from dgprf import _native as N  # noqa: E402
from dgprf import engine as E  # noqa: E402
from dgprf.data import regression_data  # noqa: E402

C = int(sys.argv[1]) if len(sys.argv) > 1 else 64
dev = torch.device("cuda", 0)
X, Y, _ = regression_data(200, 8, seed=0, device=dev)
spec = E.ModelSpec(8, 1, [N.RBF] * 3, [1024] * 3, [8, 8, 1])
e1 = E.Engine(spec, 1, seed=5)
E.normal(None, N.RNG_Z, out=e1.z)
E.normal(None, N.RNG_W, out=e1.theta)
eC = E.Engine(spec, C, seed=5)
eC.z.copy_(e1.z)
eC.hyp.copy_(e1.hyp)
eC.theta.copy_(e1.theta.expand(C, -1))
for e in (e1, eC):
    e.init_moments()
    e.build_omega()
print("slices per layer: 1 chain", list(e1.layout.ns[:3]), f"{C} chains", list(eC.layout.ns[:3]))
g1 = e1.grad(X, Y, 1e6)
gC = eC.grad(X, Y, 1e6)
err = ((gC - g1).abs().max() / g1.abs().max()).item()
print(f"max |g_C - g_1| / max |g_1| = {err:.3e}")
assert err < 1e-5
