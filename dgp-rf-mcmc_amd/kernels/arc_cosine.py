"""ARCKernel — mirror of the reference's kernels/arc_cosine.py:5-56 (degree 1 only)."""
from ._base import _RFKernel


class ARCKernel(_RFKernel):
    kernel_type = "ARC"

    def __init__(self, n_feature=1, amplitude=1., length_scale=None, trainable=True, is_ard=False,
                 degree=1, name=None):
        super().__init__(name=name)
        self.kernel_type = "ARC"
        if degree == 1:  # kernels/arc_cosine.py:13-16
            self.degree = degree
        else:
            raise NotImplementedError
        self._init_hyper(n_feature, amplitude, length_scale, trainable, is_ard)
