"""Mirror of the reference's utils.py:1-74 (layer stacks, log_gaussian, cyclical_step_rate).

Inside a DGP_RF the stack is executed by the fused HIP forward (dgprf_forward); the sequential
path below is used only for stand-alone BNNs built from layer lists.
"""
import numpy as np
import torch

from dgprf.module import Module
from layers import ARCLayer, GPLayer, RBFLayer


class BNN_from_list(Module):
    def __init__(self, layer_list, name=None):
        super().__init__(name=name)
        self.layers = layer_list
        self._model = None  # set by DGP_RF: run the fused device forward

    def __call__(self, X, allow_gradient_from_W=True):
        if self._model is not None:
            return self._model._fused_forward(X)
        for layer in self.layers:
            if isinstance(layer, GPLayer):
                X = layer(X, allow_gradient_from_W=allow_gradient_from_W)
            else:
                X = layer(X)
        return X

    def set_random_fixed(self, state):
        for layer in self.layers:
            if isinstance(layer, RBFLayer) or isinstance(layer, ARCLayer):
                assert hasattr(layer, 'random_fixed'), "Layers cannot set random_fixed!"
                layer.set_random_fixed(state)
        if self._model is not None:
            self._model._rebind_z()

    @property
    def gp_layers(self):
        return (self.layers[2 * l + 1] for l in range(len(self.layers) // 2))


class BNN_from_list_input_cat(BNN_from_list):
    def __init__(self, layer_list, name=None):
        super().__init__(layer_list, name=name)

    def __call__(self, X, allow_gradient_from_W=True):
        """utils.py:32-44: RF layers 2..L see [F | X]; first and last layer called plainly."""
        if self._model is not None:
            return self._model._fused_forward(X)
        total_layers = len(self.layers)
        Xd = X
        F = X
        for l, layer in enumerate(self.layers):
            if l == 0 or l == total_layers - 1:
                F = layer(F)
            else:
                if isinstance(layer, GPLayer):
                    F = layer(F, allow_gradient_from_W=allow_gradient_from_W)
                else:  # input concatenate
                    F = torch.cat([F, torch.as_tensor(Xd, dtype=torch.float32, device=F.device)],
                                  dim=-1)
                    F = layer(F)
        return F


def log_gaussian(x, mean=0., var=1.):
    """-0.5 (log 2pi + log var + (x - mean)^2 / var)   (utils.py:46-47)."""
    x = torch.as_tensor(x, dtype=torch.float32)
    var = torch.as_tensor(var, dtype=torch.float32, device=x.device)
    mean = torch.as_tensor(mean, dtype=torch.float32, device=x.device)
    return -0.5 * (np.log(2. * np.pi) + torch.log(var) + torch.square(x - mean) / var)


def cyclical_step_rate(step_index, cycle_length, schedule='cosine', min_value=0.001):
    """Step-rate schedule of utils.py:49-73, evaluated in float32 like the TF ops.

    :param step_index: current step (i.e. batch index), from 1
    :return: (step_rate, is_end_of_period_iteration)
    The same schedule runs on the device inside graph-captured sampling (DGPRF_SCHED_CYCLICAL).
    """
    step_index = int(step_index)
    if step_index <= 0:
        raise ValueError('Step index should be larger than zero!')
    f32 = np.float32
    frac = f32((step_index - 1) % cycle_length) / f32(cycle_length)
    if schedule == 'cosine':
        step_rate = f32(min_value) + f32(1.0 - min_value) * f32(0.5) * (
            np.cos(f32(np.pi) * frac) + f32(1.0))
    elif schedule == 'glide':
        step_rate = f32(min_value) + f32(1.0 - min_value) * (np.exp(-frac / (f32(1.0) - frac)))
    elif schedule == 'flat':
        step_rate = f32(1.0)
    else:
        raise NotImplementedError
    is_end_of_period_iteration = (step_index % cycle_length) == 0
    return f32(step_rate), bool(is_end_of_period_iteration)
