"""Minimal stand-in for tf.Module / tf.Variable used by the reference's API surface.

State lives in torch tensors on the HIP device; a tensor carries `trainable` like a tf.Variable
(kernels/RBF.py:39-41, likelihoods/gaussian.py:12, layers/GP_weight_layers.py:9).
"""
import torch


def default_device():
    """HIP device when visible; host tensors only for objects that never compute (kernels and
    likelihood hyper-parameters before they are bound to a model)."""
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
        else torch.device("cpu")


def variable(value, trainable=True, name=None, dev=None):
    t = torch.as_tensor(value, dtype=torch.float32).to(dev or default_device()).clone()
    t.trainable = bool(trainable)
    t.var_name = name
    return t


def rebind(t, view):
    """Copy t's value into `view` (a slice of packed engine storage) and carry its flags."""
    view.copy_(t.detach().reshape(view.shape).to(view.device))
    view.trainable = getattr(t, "trainable", True)
    view.var_name = getattr(t, "var_name", None)
    return view


class Module:
    """tf.Module-like: name + trainable_variables gathered from attributes in definition order."""

    def __init__(self, name=None):
        self.name = name

    def _submodules_and_vars(self):
        for k, v in vars(self).items():
            if k.startswith("_"):
                continue
            yield v

    @property
    def trainable_variables(self):
        out, seen = [], set()

        def visit(v):
            if torch.is_tensor(v):
                if getattr(v, "trainable", False) and id(v) not in seen:
                    seen.add(id(v))
                    out.append(v)
            elif isinstance(v, Module):
                for x in v._submodules_and_vars():
                    visit(x)
            elif isinstance(v, (list, tuple)):
                for x in v:
                    visit(x)

        for v in self._submodules_and_vars():
            visit(v)
        return tuple(out)
