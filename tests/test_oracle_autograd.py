"""The oracle's analytic backward (the restatement of tape.gradient, models/dgp.py:194-198)
against torch-CPU autograd of an independent forward, and finite differences."""
import numpy as np
import pytest
import torch

from oracle import dgp_oracle as O



def torch_U(p, Ws, X, Y, N):
    X = torch.as_tensor(X)
    F = X
    for l in range(p.L):
        Xin = F if (l == 0 or not p.input_cat) else torch.cat([F, X], dim=-1)
        om = torch.exp(torch.as_tensor(p.log_inv_ls[l]))[:, None] * torch.as_tensor(p.z[l]) \
            + torch.as_tensor(p.mean[l])[:, None]
        A = Xin @ om
        amp = np.exp(float(p.log_amp[l]))
        if p.kinds[l] == "RBF":
            Phi = amp / np.sqrt(p.n_rf[l]) * torch.cat([torch.cos(A), torch.sin(A)], dim=-1)
        else:
            Phi = np.sqrt(2.0) * amp / np.sqrt(p.n_rf[l]) * torch.relu(A)
        F = Phi @ Ws[l]
    Yt = torch.as_tensor(Y)
    if p.likelihood == "gaussian":
        var = float(np.exp(p.lik_log_var))
        lp = torch.sum(-0.5 * (np.log(2 * np.pi) + np.log(var) + (Yt - F) ** 2 / var), dim=-1)
    else:
        lp = -torch.nn.functional.cross_entropy(F, Yt[:, 0].long(), reduction="none")
    prior = sum(torch.sum(-0.5 * (np.log(2 * np.pi) + w ** 2)) for w in Ws)
    return -(prior / N + torch.sum(lp) / X.shape[0])


CASES = [
    (["RBF"], [17], [3], 2, 3, False, "gaussian"),
    (["RBF", "RBF", "RBF"], [20, 20, 20], [4, 4, 1], 5, 1, False, "gaussian"),
    (["ARC", "ARC"], [30, 25], [5, 2], 3, 2, False, "gaussian"),
    (["RBF", "ARC", "RBF"], [12, 18, 10], [3, 4, 4], 6, 4, True, "softmax"),
]


@pytest.mark.parametrize("case", CASES)
def test_grad_matches_autograd(case):
    kinds, n_rf, n_gp, d_in, d_out, cat, lik = case
    rng = np.random.default_rng(7)
    p = O.Params(d_in, d_out, n_rf, n_gp, kinds, lik, cat, rng=rng,
                 log_amp=[0.2] * len(kinds), lik_log_var=np.log(0.3))
    B, N = 23, 400
    X = rng.standard_normal((B, d_in))
    Y = rng.standard_normal((B, d_out)) if lik == "gaussian" else \
        rng.integers(0, d_out, (B, 1)).astype(float)
    Ws = [torch.tensor(w, requires_grad=True) for w in p.W]
    Ut = torch_U(p, Ws, X, Y, N)
    Ut.backward()
    assert np.isclose(Ut.item(), O.U(p, X, Y, N), rtol=1e-12)
    g = O.grad_W(p, X, Y, N)
    for l in range(p.L):
        np.testing.assert_allclose(g[l], Ws[l].grad.numpy(), rtol=1e-9, atol=1e-12)


def test_grad_finite_difference():
    rng = np.random.default_rng(3)
    p = O.Params(2, 1, [9, 7], [2, 1], ["RBF", "ARC"], "gaussian", False, rng=rng)
    X, Y = rng.standard_normal((11, 2)), rng.standard_normal((11, 1))
    g = O.grad_W(p, X, Y, 50)
    eps = 1e-6
    for l, (i, j) in [(0, (3, 1)), (0, (10, 0)), (1, (2, 0)), (1, (5, 0))]:
        w0 = p.W[l][i, j]
        p.W[l][i, j] = w0 + eps
        up = O.U(p, X, Y, 50)
        p.W[l][i, j] = w0 - eps
        dn = O.U(p, X, Y, 50)
        p.W[l][i, j] = w0
        assert np.isclose((up - dn) / (2 * eps), g[l][i, j], rtol=1e-5, atol=1e-9)


def test_update_matches_reference_formula():
    """m <- b m - h N g + sqrt(2(1-b) T M) xi; W <- W + h m / M  (models/dgp.py:206-216)."""
    rng = np.random.default_rng(0)
    W, m, g, xi = (rng.standard_normal((5, 2)) for _ in range(4))
    lr, N, b, T, M = 0.02, 1000.0, 0.9, 1.0, 1.7
    W1, m1 = O.sghmc_update(W, m, g, lr, N, b, T, M, xi)
    h = np.sqrt(lr / N)
    m_exp = b * m - h * N * g + np.sqrt(2 * (1 - b) * T * M) * xi
    np.testing.assert_allclose(m1, m_exp)
    np.testing.assert_allclose(W1, W + h / M * m_exp)
    # SGLD (b = 0) ignores the old momentum; resample ignores M (Appendix A.1)
    W2, m2 = O.sghmc_update(W, m, g, lr, N, 0.0, T, M, xi, xi_resample=np.ones_like(m))
    np.testing.assert_allclose(m2, -h * N * g + np.sqrt(2 * T * M) * xi)
