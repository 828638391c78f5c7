"""Large minibatches (SURVEY.md §8d B-sweep): the row-group backward k_step_bwd_rg, which keeps
every workgroup's gW in accumulators over ceil(n_row_tiles / 16) row tiles so that the gW partial
rows stay <= 16 whatever B, against the float64 oracle (models/dgp.py:194-198 gradient,
:206-216 update).

Tolerances: gradients 2e-4 of the gradient scale (fp32 sums over up to 8192 rows in a different
order than the oracle's float64); forward 5e-5.  Row-group plan facts (rows <= 16, one group per
16 row tiles) are exact.
"""
import numpy as np
import pytest
import torch

from oracle import dgp_oracle as O
from test_gpu_parity import cpu, dev, rel_err, unpack  # noqa: F401

pytestmark = pytest.mark.gpu


def _model(kinds, n_rf, n_gp, d_in, cat, lik, seed):
    from dgprf import engine as E
    from likelihoods import Gaussian, Softmax
    from models.dgp import DGP_RF
    E.set_seed(seed)
    return DGP_RF(d_in, n_gp[-1], n_hidden_layers=len(kinds), n_rf=n_rf, n_gp=n_gp,
                  likelihood=Gaussian(variance=0.3) if lik == "gaussian" else Softmax(),
                  kernel_type_list=kinds, input_cat=cat, set_nonzero_mean=True)


def _oracle(m, kinds, n_rf, n_gp, d_in, cat, lik):
    L = len(kinds)
    with torch.no_grad():
        for l in range(L):  # nonzero means exercise the Omega offsets
            m.BNN.layers[2 * l].mean.copy_(0.1 * torch.randn_like(m.BNN.layers[2 * l].mean))
    return O.Params(d_in, n_gp[-1], n_rf, n_gp, kinds, lik, cat,
                    z=[cpu(m.BNN.layers[2 * l].z) for l in range(L)],
                    W=[cpu(w) for w in m.W_mcmc],
                    log_amp=[cpu(k.log_amplitude) for k in m.kernel_list],
                    log_inv_ls=[cpu(k.log_inv_length_scale) for k in m.kernel_list],
                    mean=[cpu(m.BNN.layers[2 * l].mean)[:, 0] for l in range(L)],
                    lik_log_var=np.log(0.3))


def _rows_off_kinks(p, kinds, X, Y, n, tau=1e-5):
    """The first n rows whose ARC-layer inner products all satisfy |A| >= tau in the float64
    oracle: a row whose relu input sits within fp32 rounding of 0 can flip sides between the GPU's
    forward and the oracle's and move the gradient by a whole feature's contribution (the same
    selection as tests/test_gpu_configs.py)."""
    _, cache = O.forward(p, X, keep=True)
    ok = np.ones(X.shape[0], dtype=bool)
    for l, k in enumerate(kinds):
        if k == "ARC":
            ok &= np.min(np.abs(cache[l][1]), axis=1) >= tau
    idx = np.nonzero(ok)[0][:n]
    assert len(idx) == n, "not enough rows away from the relu kink"
    return X[idx], Y[idx]


CASES = [
    # kinds, n_rf, n_gp, d_in, input_cat, likelihood, B      (what it exercises)
    (["RBF", "ARC", "RBF"], [64, 48, 40], [5, 3, 1], 7, False, "gaussian", 300),     # 4x4 waves, ragged group
    (["ARC", "RBF"], [2048, 300], [9, 4], 9, False, "softmax", 1000),               # 8 chunk-waves x 2 rows
    (["RBF", "RBF"], [4096, 1024], [30, 10], 40, False, "softmax", 520),             # A_1 GEMM layer, 2 out tiles
    (["RBF", "ARC"], [8192, 100], [16, 1], 16, False, "gaussian", 700),              # 2 chunks per wave, g = 1
    (["ARC", "RBF"], [64, 64], [16, 5], 40, True, "softmax", 400),                   # input_cat, wide d, 16 rows
    (["RBF"] * 3, [1024] * 3, [8, 8, 1], 8, False, "gaussian", 8192),                # config 2 at B = 8192 (row-wave)
    (["ARC"] * 3, [2048] * 3, [9, 9, 1], 9, False, "gaussian", 2048),                # config 3 shape, row-wave, 8 chunks
    (["RBF", "ARC"], [1000, 200], [7, 3], 5, False, "softmax", 4000),                # row-wave, ragged R and groups
]


@pytest.mark.parametrize("case", range(len(CASES)))
def test_row_group_gradient_matches_oracle(dev, case):
    kinds, n_rf, n_gp, d_in, cat, lik, B = CASES[case]
    m = _model(kinds, n_rf, n_gp, d_in, cat, lik, 40 + case)
    p = _oracle(m, kinds, n_rf, n_gp, d_in, cat, lik)
    eng = m._engine
    pl = eng.plan_ws(B)[0]
    n_rt = (B + 15) // 16
    assert pl.n_row_tiles == n_rt and pl.rt_per_group == (n_rt + 15) // 16 > 1
    assert pl.n_gw_rows == -(-n_rt // pl.rt_per_group) <= 16 and pl.n_rt_pad == 16
    rng = np.random.default_rng(case)
    X = rng.standard_normal((2 * B, d_in))
    Y = rng.standard_normal((2 * B, n_gp[-1])) if lik == "gaussian" else \
        rng.integers(0, n_gp[-1], (2 * B, 1)).astype(float)
    X, Y = _rows_off_kinks(p, kinds, X, Y, B)
    N_ = 50_000
    G = unpack(eng, eng.grad(X, Y, N_))
    ref = O.grad_W(p, X, Y, N_)
    for l in range(len(kinds)):
        assert rel_err(G[l], ref[l]) < 2e-4, (case, l, rel_err(G[l], ref[l]))
    # the step's log p rows (written by the last layer's backward) feed U
    assert rel_err(cpu(m.BNN(X)), O.forward(p, X)) < 5e-5


def test_row_group_step_and_graph_replay(dev):
    """At B = 2048 the graph-replayed steps equal eager steps bit for bit (the row-group sums run in
    a fixed order), and one injected-noise step matches the oracle update."""
    from dgprf import engine as E
    from likelihoods import Gaussian
    from models.regression_model import RegressionDGP
    mk = lambda: RegressionDGP(6, 1, n_hidden_layers=2, n_rf=[256, 128], n_gp=[4, 1],
                               likelihood=Gaussian(variance=0.2))
    E.set_seed(77)
    a = mk()
    E.set_seed(77)
    b = mk()
    n, B = 20_480, 2048
    X = torch.randn(n, 6, device=dev)
    Y = torch.randn(n, 1, device=dev)
    for mm in (a, b):
        mm.precond_update(None, n, precond_type="identity")
    b._engine.mom.copy_(a._engine.mom)
    a.run_sgmcmc(X, Y, n, 12, batch_size=B, lr=0.01, momentum_decay=0.9, steps_per_graph=4,
                 perm_seed=2)
    for _ in range(12):
        b._engine.step(X, Y, n, 0.01, 0.9, 1.0, batch_size=B, mode=2, perm_seed=2)
    assert torch.equal(a._engine.theta, b._engine.theta)
    # one injected-noise step against the oracle update
    eng = a._engine
    p = O.Params(6, 1, [256, 128], [4, 1], ["RBF", "RBF"],
                 z=[cpu(eng.z_view(l)) for l in range(2)], W=[cpu(w) for w in a.W_mcmc],
                 log_inv_ls=[cpu(k.log_inv_length_scale) for k in a.kernel_list],
                 lik_log_var=np.log(0.2))
    rng = np.random.default_rng(5)
    Xb = rng.standard_normal((B, 6))
    Yb = rng.standard_normal((B, 1))
    m0 = unpack(eng, eng.mom)
    xi = [rng.standard_normal(w.shape) for w in p.W]
    xt = torch.zeros(1, eng.layout.w_total, dtype=torch.float32)
    for l in range(2):
        o = eng.layout.w_off[l]
        xt[0, o:o + xi[l].size] = torch.as_tensor(xi[l].reshape(-1), dtype=torch.float32)
    eng.step(Xb, Yb, n, 0.01, 0.9, 1.0, xi=xt.to(dev))
    g = O.grad_W(p, Xb, Yb, n)
    for l in range(2):
        W1, m1 = O.sghmc_update(p.W[l], m0[l], g[l], 0.01, n, 0.9, 1.0, 1.0, xi[l])
        assert rel_err(cpu(eng.W_view(l)), W1) < 1e-5
        assert rel_err(cpu(eng.mom_view(l)), m1) < 2e-4
