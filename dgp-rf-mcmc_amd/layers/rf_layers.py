"""RBFLayer / ARCLayer — mirror of the reference's layers/rf_layers.py:5-94.

Stand-alone calls run two HIP kernels: dgprf_rf_omega (Omega = exp(log_inv_ls) z + mean, c) and
dgprf_rf_features (Phi = c[cos(X Omega) | sin(X Omega)] or c relu(X Omega)).  Inside a DGP_RF the
whole stack runs fused (dgprf_forward / dgprf_sghmc_step) on the same packed storage.
"""
import ctypes

import torch

from dgprf import _native as N
from dgprf import engine as E
from dgprf.module import Module, variable
from kernels import ARCKernel, RBFKernel


class _RFLayer(Module):
    _kind = None

    def _init_common(self, kernel, out_feature, random_fixed, set_nonzero_mean):
        self.kernel = kernel
        self.in_feature = int(kernel.n_feature)
        self.out_feature = int(out_feature)
        self.random_fixed = random_fixed
        if random_fixed:  # when training (rf_layers.py:21-22)
            self.z = E.normal((self.in_feature, self.out_feature), N.RNG_Z)
            self.z.trainable = False
        self.set_nonzero_mean = set_nonzero_mean
        # mean is a Variable only when set_nonzero_mean (rf_layers.py:23-27)
        self.mean = variable(torch.zeros(self.in_feature, 1), trainable=bool(set_nonzero_mean),
                             name="mean", dev=E.device())

    def _omega(self):
        """(Omega [d, R], c [1]) for this call; fresh z if not random_fixed (rf_layers.py:39-41)."""
        dev = E.device()
        z = self.z if self.random_fixed else E.normal((self.in_feature, self.out_feature), N.RNG_Z)
        om = torch.empty(self.in_feature, self.out_feature, dtype=torch.float32, device=dev)
        c = torch.empty(1, dtype=torch.float32, device=dev)
        lis = E.as_device(self.kernel.log_inv_length_scale.detach().reshape(-1), dev)
        la = E.as_device(self.kernel.log_amplitude.detach().reshape(1), dev)
        mean = E.as_device(self.mean.detach().reshape(-1), dev)
        N.call("dgprf_rf_omega", self._kind, self.in_feature, self.out_feature, E.ptr(z),
               E.ptr(lis), E.ptr(mean), E.ptr(la), E.ptr(om), E.ptr(c), E.stream())
        return om, c, (z, lis, la, mean)

    def __call__(self, X):
        """X [B, in_feature] -> Phi [B, n_rf]."""
        dev = E.device()
        X = E.as_device(X, dev)
        if X.dim() != 2 or X.shape[1] != self.in_feature:
            raise ValueError(f"X must be [B, {self.in_feature}], got {tuple(X.shape)}")
        om, c, keep = self._omega()
        phi = torch.empty(X.shape[0], self.n_rf, dtype=torch.float32, device=dev)
        N.call("dgprf_rf_features", self._kind, E.ptr(X), X.shape[0], self.in_feature, E.ptr(om),
               self.out_feature, E.ptr(c), E.ptr(phi), E.stream())
        return phi

    def set_random_fixed(self, state):
        self.random_fixed = state
        if state and not hasattr(self, "z"):
            self.z = E.normal((self.in_feature, self.out_feature), N.RNG_Z)
            self.z.trainable = False


class RBFLayer(_RFLayer):
    _kind = N.RBF

    def __init__(self, kernel, out_feature, random_fixed=True, set_nonzero_mean=False, name=None):
        """:param kernel: RBFKernel; :param out_feature: number of sampled Omegas (rf_layers.py:6-27)"""
        super().__init__(name=name)
        assert isinstance(kernel, RBFKernel), "Input kernel is not RBF!"
        self._init_common(kernel, out_feature, random_fixed, set_nonzero_mean)
        self.n_rf = 2 * self.out_feature


class ARCLayer(_RFLayer):
    _kind = N.ARC

    def __init__(self, kernel, out_feature, random_fixed=True, set_nonzero_mean=False, name=None):
        """:param kernel: ARC-cosine kernel; :param out_feature: number of sampled Omegas (:52-73)"""
        super().__init__(name=name)
        assert isinstance(kernel, ARCKernel), "Input kernel is not ARC!"
        self._init_common(kernel, out_feature, random_fixed, set_nonzero_mean)
        self.n_rf = self.out_feature
