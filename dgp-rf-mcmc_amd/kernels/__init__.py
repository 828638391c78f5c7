from .RBF import RBFKernel
from .arc_cosine import ARCKernel
