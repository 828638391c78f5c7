"""The hot path as torch operators (torch.ops.dgprf, libdgprf_torch.so over the C-ABI): the
dispatcher sees them, they run on torch's current HIP stream, and torch.cuda.graph captures them.

  sghmc_step_     DGP_RF.sgmcmc_update (models/dgp.py:184-216)
  potential_grad  U + tape.gradient (models/dgp.py:161-182, 194-198)
  forward         BNN(X) + log p / se + online LSE (utils.py:10-44, models/regression_model.py:33-50)
  lse_finalize    experiments/utils_training.py:79-85
Bit-exact checks: a captured step replayed K times equals K eager op calls (same Philox counters,
same kernels); the oracle parity of each op is the rest of the GPU suite, which calls them through
dgprf.engine.
"""
import numpy as np
import pytest
import torch

from test_gpu_parity import cpu, dev  # noqa: F401

pytestmark = pytest.mark.gpu


def _small_model(seed):
    from dgprf import engine as E
    from likelihoods import Gaussian
    from models.regression_model import RegressionDGP
    E.set_seed(seed)
    m = RegressionDGP(3, 1, n_hidden_layers=2, n_rf=[64, 48], n_gp=[4, 1],
                      likelihood=Gaussian(variance=0.1), kernel_type_list=["RBF", "ARC"])
    m.precond_update(None, 1000, precond_type="identity")
    return m


def test_ops_registered_with_dispatcher(dev):
    from dgprf import _native as N
    ops = N.torch_ops()
    for name in ("sghmc_step_", "potential_grad", "forward", "lse_finalize"):
        schema = str(getattr(ops, name).default._schema)
        assert schema.startswith(f"dgprf::{name}("), schema
    assert "Tensor(a!) theta" in str(ops.sghmc_step_.default._schema)


def test_sghmc_step_op_captured_by_torch_cuda_graph(dev):
    """torch.cuda.graph around Engine.step (torch.ops.dgprf.sghmc_step_, device Philox noise keyed
    on the device step counter): 4 replays == 4 eager steps, bit for bit, and the step counter
    advanced by 4 in both."""
    m = _small_model(3)
    eng = m._engine
    rng = np.random.default_rng(1)
    X = torch.as_tensor(rng.standard_normal((50, 3)), dtype=torch.float32, device=dev)
    Y = torch.as_tensor(rng.standard_normal((50, 1)), dtype=torch.float32, device=dev)
    eng.build_omega()
    state = [t.clone() for t in (eng.theta, eng.mom, eng.step_ctr)]
    for _ in range(4):
        eng.step(X, Y, 1000, 0.01, 0.9, 1.0, build=False)
    eager = (eng.theta.clone(), eng.mom.clone(), eng.step_ctr.clone())
    for t, s in zip((eng.theta, eng.mom, eng.step_ctr), state):
        t.copy_(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        eng.step(X, Y, 1000, 0.01, 0.9, 1.0, build=False)
    # capture does not execute: the state is still the restored one
    assert torch.equal(eng.step_ctr, state[2])
    for _ in range(4):
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(eng.theta, eager[0]) and torch.equal(eng.mom, eager[1])
    assert int(eng.step_ctr.item()) == int(state[2].item()) + 4 == int(eager[2].item())


def test_forward_and_finalize_ops_captured_by_torch_cuda_graph(dev):
    """torch.cuda.graph around PredictiveLSE.add_sample (torch.ops.dgprf.forward folding into the
    LSE accumulators): two replays fold the same sample twice, equal to two eager folds; then
    torch.ops.dgprf.lse_finalize of those accumulators gives LL = mean(log p) (two identical samples:
    LSE - log 2 = log p) and RMSE = sqrt(mean se)."""
    from dgprf.predictive import PredictiveLSE
    m = _small_model(4)
    eng = m._engine
    rng = np.random.default_rng(2)
    Xt = torch.as_tensor(rng.standard_normal((333, 3)), dtype=torch.float32, device=dev)
    Yt = torch.as_tensor(rng.standard_normal((333, 1)), dtype=torch.float32, device=dev)
    eng.build_omega()
    ref = eng.forward(Xt, Yt, logp=True, se=True, build=False)
    eager = PredictiveLSE(eng, Xt, Yt)
    eager.add_sample(build=False)
    eager.add_sample(build=False)
    acc = PredictiveLSE(eng, Xt, Yt)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        acc.add_sample(build=False)
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    for k in ("m", "s", "e"):
        assert torch.equal(getattr(acc, k), getattr(eager, k)), k
    acc.S = 2
    ll, rmse = acc.finalize()
    lp, se = cpu(ref["logp"][0]).astype(np.float64), cpu(ref["se"][0]).astype(np.float64)
    assert abs(ll - lp.mean()) < 1e-5 * max(1.0, abs(lp.mean()))
    assert abs(rmse - np.sqrt(se.mean())) < 1e-5 * np.sqrt(se.mean())
