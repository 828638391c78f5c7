"""Gaussian likelihood — mirror of the reference's likelihoods/gaussian.py:6-25.

Inside a DGP_RF the likelihood and its gradient are evaluated in libdgprf's kernels (the step
backward prologue and dgprf_forward); log_prob here is the stand-alone tensor utility."""
import numpy as np
import torch

from dgprf.module import Module, variable


class Gaussian(Module):
    def __init__(self, variance=0.1, trainable=True):
        """:param variance: sigma^2, noise variance should be greater than 0."""
        super().__init__()
        self.lik_log_var = variable(np.log(np.float32(variance)), trainable, "lik_log_var")

    @property
    def variance(self):
        return torch.exp(self.lik_log_var)

    def log_prob(self, F, Y):
        """sum over the last axis of log N(Y | F, sigma^2)."""
        from utils import log_gaussian
        F = torch.as_tensor(F, dtype=torch.float32)
        Y = torch.as_tensor(Y, dtype=torch.float32, device=F.device)
        return torch.sum(log_gaussian(Y, mean=F, var=self.variance.to(F.device)), dim=-1)
