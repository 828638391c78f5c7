"""GPLayer — mirror of the reference's layers/GP_weight_layers.py:4-20 (F = Phi W on the device)."""
import numpy as np
import torch

from dgprf import _native as N
from dgprf import engine as E
from dgprf.module import Module


class GPLayer(Module):
    def __init__(self, in_feature, out_feature, name=None):
        super().__init__(name=name)
        self.in_feature = int(in_feature)
        self.out_feature = int(out_feature)
        self.W = E.normal((self.in_feature, self.out_feature), N.RNG_W)  # W ~ N(0, 1), :9
        self.W.trainable = True
        self.W.var_name = "GP_layer_W"

    def __call__(self, X, allow_gradient_from_W=True):
        """F = X W (:11-15).  Gradients are analytic in libdgprf, so allow_gradient_from_W only
        matters to the reference's tape and is accepted for signature compatibility."""
        dev = E.device()
        X = E.as_device(X, dev)
        if X.dim() != 2 or X.shape[1] != self.in_feature:
            raise ValueError(f"X must be [B, {self.in_feature}], got {tuple(X.shape)}")
        F = torch.empty(X.shape[0], self.out_feature, dtype=torch.float32, device=dev)
        N.call("dgprf_gp_matmul", E.ptr(X), X.shape[0], self.in_feature, E.ptr(self.W),
               self.out_feature, E.ptr(F), E.stream())
        return F

    def assign_W(self, W_value):
        """W.assign(value) (:17-20); accepts numpy arrays or tensors."""
        if not torch.is_tensor(W_value):
            W_value = torch.as_tensor(np.asarray(W_value, dtype=np.float32))
        if tuple(W_value.shape) != tuple(self.W.shape):
            raise ValueError(f"assign_W: shape {tuple(W_value.shape)} != {tuple(self.W.shape)}")
        with torch.no_grad():
            self.W.copy_(W_value.to(self.W.device, torch.float32))
