"""RBFKernel — mirror of the reference's kernels/RBF.py:5-53 (hyper-parameters only; the RF
feature map that uses them runs in libdgprf.so)."""
from ._base import _RFKernel


class RBFKernel(_RFKernel):
    kernel_type = "RBF"

    def __init__(self, n_feature=1, amplitude=1., length_scale=None, trainable=True, is_ard=False,
                 name=None):
        """k(x, y) = amplitude**2 * exp(-||x - y||**2 / (2 * length_scale**2))"""
        super().__init__(name=name)
        self.kernel_type = "RBF"
        self._init_hyper(n_feature, amplitude, length_scale, trainable, is_ard)
