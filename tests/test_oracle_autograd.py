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


# ----------------------------------------------------------------------------- full Bayes
def torch_U_full(p, t, X, Y, N, tr):
    """Independent torch forward of U with full_bayesian=True (models/dgp.py:175-181) over the
    leaf tensors in `t` (W, log_amp, log_inv_ls, mean, lik_log_var)."""
    X = torch.as_tensor(X)
    F = X
    for l in range(p.L):
        Xin = F if (l == 0 or not p.input_cat) else torch.cat([F, X], dim=-1)
        lis = t["log_inv_ls"][l]
        if lis.dim() == 0:
            lis = lis.expand(p.d[l])
        om = torch.exp(lis)[:, None] * torch.as_tensor(p.z[l]) + t["mean"][l][:, None]
        A = Xin @ om
        amp = torch.exp(t["log_amp"][l])
        if p.kinds[l] == "RBF":
            Phi = amp / np.sqrt(p.n_rf[l]) * torch.cat([torch.cos(A), torch.sin(A)], dim=-1)
        else:
            Phi = np.sqrt(2.0) * amp / np.sqrt(p.n_rf[l]) * torch.relu(A)
        F = Phi @ t["W"][l]
    Yt = torch.as_tensor(Y)
    if p.likelihood == "gaussian":
        var = torch.exp(t["lik_log_var"])
        lp = torch.sum(-0.5 * (np.log(2 * np.pi) + torch.log(var) + (Yt - F) ** 2 / var), dim=-1)
    else:
        lp = -torch.nn.functional.cross_entropy(F, Yt[:, 0].long(), reduction="none")
    lg = lambda v: torch.sum(-0.5 * (np.log(2 * np.pi) + v ** 2))
    prior = sum(lg(w) for w in t["W"])
    for l in range(p.L):
        if tr.kernel:
            prior = prior + lg(t["log_amp"][l]) + lg(t["log_inv_ls"][l])
        if tr.mean:
            prior = prior + lg(t["mean"][l])
    if tr.lik and p.likelihood == "gaussian":
        prior = prior + lg(t["lik_log_var"])
    return -(prior / N + torch.sum(lp) / X.shape[0])


FULL_CASES = [
    (["RBF"], [17], [3], 2, 3, False, "gaussian", O.Trainable()),
    (["RBF", "RBF", "RBF"], [20, 20, 20], [4, 4, 1], 5, 1, False, "gaussian",
     O.Trainable(mean=True)),
    (["ARC", "ARC"], [30, 25], [5, 2], 3, 2, False, "gaussian", O.Trainable(ard=[False, True])),
    (["RBF", "ARC", "RBF"], [12, 18, 10], [3, 4, 4], 6, 4, True, "softmax",
     O.Trainable(mean=True, ard=[True, False, True])),
    (["RBF", "RBF"], [16, 16], [3, 2], 4, 2, False, "gaussian", O.Trainable(kernel=False)),
]


@pytest.mark.parametrize("case", FULL_CASES)
def test_full_bayes_grad_matches_autograd(case):
    kinds, n_rf, n_gp, d_in, d_out, cat, lik, tr = case
    rng = np.random.default_rng(11)
    L = len(kinds)
    d = O.layer_widths(d_in, n_gp, cat)
    lis = [O.init_log_inv_ls(d[l]) + (0.1 * rng.standard_normal(d[l])
                                      if (tr.ard is None or tr.ard[l]) else 0.0) for l in range(L)]
    p = O.Params(d_in, d_out, n_rf, n_gp, kinds, lik, cat, rng=rng,
                 log_amp=[0.1 * rng.standard_normal() for _ in range(L)], log_inv_ls=lis,
                 mean=[0.1 * rng.standard_normal(d[l]) for l in range(L)],
                 lik_log_var=np.log(0.3))
    B, N = 23, 400
    X = rng.standard_normal((B, d_in))
    Y = rng.standard_normal((B, d_out)) if lik == "gaussian" else \
        rng.integers(0, d_out, (B, 1)).astype(float)
    leaf = lambda a: torch.tensor(np.asarray(a, dtype=np.float64), requires_grad=True)
    t = {"W": [leaf(w) for w in p.W], "log_amp": [leaf(a) for a in p.log_amp],
         "log_inv_ls": [leaf(p.log_inv_ls[l] if (tr.ard is None or tr.ard[l])
                             else p.log_inv_ls[l][0]) for l in range(L)],
         "mean": [leaf(m) for m in p.mean], "lik_log_var": leaf(p.lik_log_var)}
    Ut = torch_U_full(p, t, X, Y, N, tr)
    Ut.backward()
    assert np.isclose(Ut.item(), O.U_full(p, X, Y, N, tr), rtol=1e-12)
    g = O.grad_full(p, X, Y, N, tr)
    for l in range(L):
        np.testing.assert_allclose(g["W"][l], t["W"][l].grad.numpy(), rtol=1e-9, atol=1e-12)
        if tr.kernel:
            for name in ("log_amp", "log_inv_ls"):
                np.testing.assert_allclose(g[name][l], t[name][l].grad.numpy(), rtol=1e-9,
                                           atol=1e-12)
        else:
            assert g["log_amp"][l] is None and g["log_inv_ls"][l] is None
        if tr.mean:
            np.testing.assert_allclose(g["mean"][l], t["mean"][l].grad.numpy(), rtol=1e-9,
                                       atol=1e-12)
    if lik == "gaussian":
        np.testing.assert_allclose(g["lik_log_var"], t["lik_log_var"].grad.numpy(), rtol=1e-9,
                                   atol=1e-12)


def test_full_bayes_step_reduces_to_w_only_when_nothing_else_trains():
    rng = np.random.default_rng(5)
    p = O.Params(3, 1, [10, 8], [2, 1], ["RBF", "RBF"], "gaussian", False, rng=rng)
    q = O.Params(3, 1, [10, 8], [2, 1], ["RBF", "RBF"], "gaussian", False,
                 z=p.z, W=[w.copy() for w in p.W])
    tr = O.Trainable(kernel=False, lik=False)
    X, Y = rng.standard_normal((9, 3)), rng.standard_normal((9, 1))
    keys = O.full_groups(p, tr)
    assert keys == [("W", 0), ("W", 1)]
    m = {k: rng.standard_normal(O.get_var(p, k, tr).shape) for k in keys}
    xi = {k: rng.standard_normal(O.get_var(p, k, tr).shape) for k in keys}
    M = {k: 1.3 for k in keys}
    O.sgmcmc_step_full(p, m, X, Y, 100.0, 0.01, 0.9, 1.0, M, xi, tr)
    O.sgmcmc_step(q, [m[k] for k in keys], X, Y, 100.0, 0.01, 0.9, 1.0, [1.3, 1.3],
                  [xi[k] for k in keys])
    for l in range(2):
        np.testing.assert_allclose(p.W[l], q.W[l], rtol=1e-12)
