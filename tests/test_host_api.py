"""Host-side behaviour of the API mirror that needs no GPU: constructor validation raises the
reference's exception types before any device work, and the product refuses to compute without
a HIP device (no CPU fallback)."""
import numpy as np
import pytest
import torch

from kernels import ARCKernel, RBFKernel
from likelihoods import Gaussian, Softmax
from utils import cyclical_step_rate, log_gaussian


def test_kernel_init_matches_reference():
    k = RBFKernel(n_feature=8, is_ard=True)
    assert k.kernel_type == "RBF" and k.is_ard
    assert torch.allclose(k.length_scale.cpu(), torch.full((8,), np.sqrt(8.0)))
    assert float(k.log_amplitude) == 0.0
    k1 = RBFKernel(n_feature=1, is_ard=True)
    assert k1.log_inv_length_scale.cpu().tolist() == [0.0]  # mcycle notebook cell 5
    a = ARCKernel(n_feature=3, is_ard=True)
    assert a.kernel_type == "ARC" and a.degree == 1


def test_kernel_errors():
    with pytest.raises(NotImplementedError):
        ARCKernel(n_feature=2, degree=2)           # kernels/arc_cosine.py:13-16
    with pytest.raises(ValueError):
        RBFKernel(n_feature=2, length_scale=np.ones((2, 2)))  # kernels/RBF.py:19-20
    with pytest.raises(ValueError):
        RBFKernel(n_feature=3, length_scale=np.ones(2))      # kernels/RBF.py:26-27
    k = RBFKernel(n_feature=3, length_scale=np.ones(3), is_ard=False)  # vector -> ARD
    assert k.is_ard
    k = RBFKernel(n_feature=3, length_scale=2.0, is_ard=False)
    assert not k.is_ard


def test_trainable_variables():
    k = RBFKernel(n_feature=2, trainable=False)
    assert len(k.trainable_variables) == 0
    assert len(RBFKernel(n_feature=2).trainable_variables) == 2
    assert len(Gaussian(trainable=True).trainable_variables) == 1
    assert len(Softmax().trainable_variables) == 0
    assert np.isclose(float(Gaussian(variance=0.01).variance), 0.01)


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU refusal")
def test_no_cpu_fallback():
    from layers import RBFLayer
    from models.regression_model import RegressionDGP
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        RBFLayer(RBFKernel(n_feature=2, is_ard=True), 10)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        RegressionDGP(2, 1, n_hidden_layers=1, n_rf=10, n_gp=1)


def test_model_config_errors_before_device_work():
    from models.dgp import DGP_RF
    with pytest.raises(AssertionError, match="random feature"):
        DGP_RF(3, 1, n_hidden_layers=2, n_rf=[10, 10, 10], n_gp=[2, 1])
    with pytest.raises(AssertionError, match="hidden GP"):
        DGP_RF(3, 1, n_hidden_layers=2, n_rf=10, n_gp=[2, 1, 1])
    with pytest.raises(AssertionError, match="Kernel type"):
        DGP_RF(3, 1, n_hidden_layers=2, n_rf=10, n_gp=[2, 1], kernel_type_list=["RBF"])
    with pytest.raises(NotImplementedError):
        DGP_RF(3, 1, n_hidden_layers=1, n_rf=10, n_gp=1, kernel_type_list=["POLY"])


def test_utils():
    x = torch.tensor([0.0, 1.0, -2.0])
    ref = -0.5 * (np.log(2 * np.pi) + np.log(0.5) + (x.numpy() - 0.3) ** 2 / 0.5)
    assert np.allclose(log_gaussian(x, mean=0.3, var=0.5).numpy(), ref)
    with pytest.raises(ValueError):
        cyclical_step_rate(0, 5)
    r, e = cyclical_step_rate(10, 5, min_value=0.0)
    assert e and abs(r - 0.5 * (np.cos(0.8 * np.pi) + 1)) < 1e-6
    lp = Gaussian(variance=0.5).log_prob(torch.zeros(4, 2), torch.ones(4, 2))
    assert np.allclose(lp.cpu().numpy(), 2 * (-0.5 * (np.log(2 * np.pi) + np.log(0.5) + 2.0)))
    sm = Softmax().log_prob(torch.tensor([[0.0, 1.0]]), torch.tensor([[1.0]]))
    assert np.isclose(float(sm), 1.0 - np.log(1 + np.e))


def test_host_stage_array_forms():
    """Per-call host batches accepted by the pinned staging ring (dgprf.engine.HostStage): numpy
    arrays, lists, CPU tensors that track gradients, bf16 CPU tensors (cast to fp32 on the host)."""
    from dgprf.engine import HostStage
    a = HostStage._host_array(torch.ones(2, 3, dtype=torch.bfloat16, requires_grad=True))
    assert a.dtype == np.float32 and a.shape == (2, 3)
    assert HostStage._host_array([[1.0, 2.0]]).shape == (1, 2)
    x = np.arange(6, dtype=np.float64).reshape(3, 2)
    assert HostStage._host_array(x) is x
    assert HostStage._host_array(torch.zeros(4)).dtype == np.float32
