"""Shared body of RBFKernel / ARCKernel (kernels/RBF.py:6-53, kernels/arc_cosine.py:6-56)."""
import numpy as np
import torch

from dgprf.module import Module, variable


class _RFKernel(Module):
    kernel_type = None

    def _init_hyper(self, n_feature, amplitude, length_scale, trainable, is_ard):
        self.n_feature = n_feature
        # initialize length scale to sqrt(d_in)   (kernels/RBF.py:15-17)
        if length_scale is None:
            length_scale = float(np.float32(n_feature) ** np.float32(0.5))
        ls = np.asarray(length_scale, dtype=np.float32)
        if ls.ndim >= 2:  # kernels/RBF.py:19-20
            raise ValueError("The length scale of RBF dim error!")
        inv = np.float32(1.0) / ls
        if inv.ndim == 0 and is_ard:  # :22-24
            inv = inv * np.ones(n_feature, dtype=np.float32)
            self.is_ard = is_ard
        elif inv.ndim == 1:  # :25-32
            if n_feature != inv.size:
                raise ValueError("The size of length scale and features do not match!")
            self.is_ard = True
            if self.is_ard != is_ard:
                print(f"Arg is_ard={is_ard} does not match the length_scale!")
                print(f"Already set is_ard={self.is_ard}")
        else:  # :33-37
            self.is_ard = False
            if self.is_ard != is_ard:
                print(f"Arg is_ard={is_ard} does not match the length_scale!")
                print(f"Already set is_ard={self.is_ard}")
        self.log_amplitude = variable(np.log(np.float32(amplitude)), trainable, "log_amplitude")
        self.log_inv_length_scale = variable(np.log(inv), trainable, "log_inv_length_scale")

    @property
    def amplitude(self):
        return torch.exp(self.log_amplitude)

    @property
    def length_scale(self):
        return 1.0 / self.inv_length_scale

    @property
    def inv_length_scale(self):
        return torch.exp(self.log_inv_length_scale)
