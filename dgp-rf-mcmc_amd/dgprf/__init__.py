"""dgprf — MI355X-native runtime behind the DGP-RF-MCMC API mirror (models/, layers/, kernels/,
likelihoods/, utils.py next to this package).  Compute goes through libdgprf.so (HIP, gfx950)."""
from . import _native  # noqa: F401
from .engine import Engine, ModelSpec, device, set_seed, lse_finalize  # noqa: F401
from .module import Module, variable  # noqa: F401

__all__ = ["Engine", "ModelSpec", "device", "set_seed", "lse_finalize", "Module", "variable"]
