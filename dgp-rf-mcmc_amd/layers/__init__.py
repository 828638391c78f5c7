from .rf_layers import RBFLayer, ARCLayer
from .GP_weight_layers import GPLayer
