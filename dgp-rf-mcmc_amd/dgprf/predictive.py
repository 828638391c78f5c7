"""Posterior-predictive accumulation over samples, chains and ranks.

Replaces the driver's `log_p.append(...)` + stack + reduce_logsumexp (experiments/utils_training.py:
63-65, 79-85): each sample's test log-likelihoods are folded into an online (max, sum) per test
point by the forward kernel itself, so no [S, N_test] matrix is materialised.  Across GPUs the
per-rank accumulators are all-gathered once (RCCL over xGMI) at finalize time.
"""
import math

import torch

from . import engine as E
from . import distributed as D


class PredictiveLSE:
    def __init__(self, engine, X_test, Y_test):
        self.eng = engine
        self.X = E.as_device(X_test, engine.dev)
        Y = E.as_device(Y_test, engine.dev)
        self.Y = Y[:, None] if Y.dim() == 1 else Y
        n = self.X.shape[0]
        C = engine.C
        self.m = torch.full((C, n), -math.inf, dtype=torch.float32, device=engine.dev)
        self.s = torch.zeros((C, n), dtype=torch.float32, device=engine.dev)
        self.gaussian = engine.spec.likelihood == 0
        self.e = torch.zeros((C, n), dtype=torch.float32, device=engine.dev) if self.gaussian \
            else None
        self.S = 0  # samples folded in (per rank, all chains)

    def _a1(self, build, omega):
        """The test set's resident X Omega_1 (wide first layer; shared by every sample, Omega_1
        being fixed across samples), or None (the A_1 GEMM runs per sample)."""
        if omega is not None:
            return None
        if build:
            self.eng.build_omega()
        return self.eng.dataset_a1(self.X)

    def add_sample(self, build=True, omega=None):
        """Score the engine's current theta (one sample per chain) on the test set."""
        a1 = self._a1(build, omega)
        if a1 is not None:
            self.eng.forward_samples(self.eng.theta[None], self.X, self.Y, (self.m, self.s, self.e),
                                     build=False, a1=a1)
        else:
            self.eng.forward(self.X, self.Y, lse=(self.m, self.s, self.e), build=build, omega=omega)
        self.S += self.eng.C

    def add_samples(self, thetas, build=True, omega=None):
        """Score S posterior samples of every chain, thetas [S, C, w_total] (or [S, w_total] for
        one chain), folded in sample order (dgprf::forward_samples: two samples per pass with the
        first layer shared for lean models)."""
        thetas = E.as_device(thetas, self.eng.dev)
        if thetas.dim() == 2:
            thetas = thetas[:, None, :]
        a1 = self._a1(build, omega)
        self.eng.forward_samples(thetas, self.X, self.Y, (self.m, self.s, self.e),
                                 build=build and a1 is None, omega=omega, a1=a1)
        self.S += thetas.shape[0] * thetas.shape[1]

    def finalize(self, y_std=1.0, group=None):
        """(test log-likelihood, RMSE) over every sample of every chain of every rank."""
        m, s, e, S = D.gather_accumulators(self.m, self.s, self.e, self.S, group)
        if e is None:
            e = torch.zeros_like(s)
        out, _ = E.lse_finalize(m, s, e, S, y_std)
        out = out.cpu()
        return float(out[0]), (float(out[1]) if self.gaussian else None)
