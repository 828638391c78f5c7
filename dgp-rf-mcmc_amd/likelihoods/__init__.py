from .softmax import Softmax
from .gaussian import Gaussian
