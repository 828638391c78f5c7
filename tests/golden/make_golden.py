"""Generate the committed golden fixtures (tests/golden/*.npz) from the float64 oracle.

Inputs (z, W, X, Y, momenta, injected noise) are drawn with numpy PCG64 from fixed seeds; the
expected outputs come from oracle/dgp_oracle.py.  TensorFlow (the reference's runtime) is not
installed here, so the reference itself cannot produce these vectors — see oracle/dgp_oracle.py
for what pins the oracle.  Re-run:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dgp-rf-mcmc_amd"))

from oracle import dgp_oracle as O  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))

# name: (kinds, n_rf, n_gp, d_in, d_out, input_cat, likelihood, B, N, seed, variance)
CASES = {
    "rbf2_gauss": (["RBF", "RBF"], [20, 36], [4, 2], 3, 2, False, "gaussian", 37, 1000, 1, 0.1),
    "arc_rbf_softmax_cat": (["ARC", "RBF"], [24, 40], [6, 3], 5, 3, True, "softmax", 50, 500, 2,
                            None),
    "mixed5": (["RBF", "ARC", "RBF", "ARC", "RBF"], [16, 24, 20, 12, 18], [3, 4, 2, 5, 1], 4, 1,
               False, "gaussian", 19, 300, 3, 0.2),
    "wide_g": (["RBF"], [40], [30], 6, 30, False, "gaussian", 21, 90, 4, 0.5),
}


def make_params(kinds, n_rf, n_gp, d_in, d_out, input_cat, lik, seed, variance, rng):
    d = O.layer_widths(d_in, n_gp, input_cat)
    L = len(kinds)
    P = [O.phi_width(k, r) for k, r in zip(kinds, n_rf)]
    z = [rng.standard_normal((d[l], n_rf[l])) for l in range(L)]
    W = [rng.standard_normal((P[l], n_gp[l])) for l in range(L)]
    log_amp = [0.1 * rng.standard_normal() for _ in range(L)]
    log_inv_ls = [O.init_log_inv_ls(d[l]) + 0.1 * rng.standard_normal(d[l]) for l in range(L)]
    mean = [0.05 * rng.standard_normal(d[l]) for l in range(L)]
    llv = np.log(variance) if variance is not None else 0.0
    return O.Params(d_in, d_out, n_rf, n_gp, kinds, lik, input_cat, z=z, W=W, log_amp=log_amp,
                    log_inv_ls=log_inv_ls, mean=mean, lik_log_var=llv)


def targets(p, B, d_out, lik, rng):
    X = rng.standard_normal((B, p.d_in))
    if lik == "gaussian":
        Y = rng.standard_normal((B, d_out))
    else:
        Y = rng.integers(0, d_out, (B, 1)).astype(np.float64)
    return X, Y


def pack_params(p, out):
    for l in range(p.L):
        out[f"z{l}"] = p.z[l]
        out[f"W{l}"] = p.W[l]
        out[f"log_amp{l}"] = np.asarray(p.log_amp[l])
        out[f"log_inv_ls{l}"] = p.log_inv_ls[l]
        out[f"mean{l}"] = p.mean[l]
    out["lik_log_var"] = np.asarray(p.lik_log_var)


def gen_case(name, spec):
    kinds, n_rf, n_gp, d_in, d_out, input_cat, lik, B, N, seed, variance = spec
    rng = np.random.default_rng(seed)
    p = make_params(kinds, n_rf, n_gp, d_in, d_out, input_cat, lik, seed, variance, rng)
    X, Y = targets(p, B, d_out, lik, rng)
    out = {"kinds": np.array([0 if k == "RBF" else 1 for k in kinds]), "n_rf": np.array(n_rf),
           "n_gp": np.array(n_gp), "dims": np.array([d_in, d_out, int(input_cat),
                                                       0 if lik == "gaussian" else 1, B, N]),
           "X": X, "Y": Y}
    pack_params(p, out)
    F, cache = O.forward(p, X, keep=True)
    for l in range(p.L):
        out[f"F{l}"] = cache[l][3]
        out[f"Phi{l}"] = cache[l][2]
    out["logp"] = O.log_prob(p, F, Y)
    if lik == "gaussian":
        out["se"] = np.mean((Y - F) ** 2, axis=-1)
    out["U"] = np.asarray(O.U(p, X, Y, N))
    out["prior_W"] = np.asarray(O.prior_W(p))
    g = O.grad_W(p, X, Y, N)
    for l in range(p.L):
        out[f"g{l}"] = g[l]
    # one SGHMC step with injected noise and injected momentum resample
    lr, beta, T = 0.01, 0.9, 1.0
    M = [1.0 + 0.5 * l for l in range(p.L)]
    m0 = [rng.standard_normal(w.shape) for w in p.W]
    xi = [rng.standard_normal(w.shape) for w in p.W]
    xr = [rng.standard_normal(w.shape) for w in p.W]
    for l in range(p.L):
        out[f"m0_{l}"], out[f"xi{l}"], out[f"xr{l}"] = m0[l], xi[l], xr[l]
    out["step_scalars"] = np.array([lr, beta, T, N])
    out["M"] = np.array(M)
    W_before = [w.copy() for w in p.W]
    m1 = O.sgmcmc_step(p, m0, X, Y, N, lr, beta, T, M, xi)
    for l in range(p.L):
        out[f"W1_{l}"], out[f"m1_{l}"] = p.W[l], m1[l]
    p.W = [w.copy() for w in W_before]
    m1r = O.sgmcmc_step(p, m0, X, Y, N, lr, beta, T, M, xi, xr)
    for l in range(p.L):
        out[f"W1r_{l}"], out[f"m1r_{l}"] = p.W[l], m1r[l]
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)


def gen_config1_sgld():
    """Config 1: 1-layer RBF n_rf=100, D=1, mcycle-shaped N=133, full batch, SGLD (beta=0),
    50 steps with injected noise."""
    from dgprf.data import mcycle_like
    X, Y, Xt, ys = mcycle_like(133, 100, seed=0)
    X, Y = X.astype(np.float64), Y.astype(np.float64)
    rng = np.random.default_rng(10)
    p = make_params(["RBF"], [100], [1], 1, 1, False, "gaussian", 10, 0.01, rng)
    p.log_amp = [np.float64(0.0)]
    p.log_inv_ls = [np.array([0.0])]
    p.mean = [np.zeros(1)]
    out = {"X": X, "Y": Y, "Xt": Xt.astype(np.float64)}
    pack_params(p, out)
    steps, lr, beta, T, N = 50, 0.01, 0.0, 1.0, 133
    m = [np.zeros_like(p.W[0])]
    xis = rng.standard_normal((steps,) + p.W[0].shape)
    traj = []
    for t in range(steps):
        m = O.sgmcmc_step(p, m, X, Y, N, lr, beta, T, [1.0], [xis[t]])
        traj.append(p.W[0].copy())
    out["xi"] = xis
    out["traj"] = np.stack(traj)
    out["step_scalars"] = np.array([lr, beta, T, N])
    lp, se = O.eval_log_likelihood_and_se(p, Xt.astype(np.float64), np.zeros((100, 1)))
    out["test_logp_final"], out["test_se_final"] = lp, se
    np.savez_compressed(os.path.join(OUT, "config1_sgld.npz"), **out)


def gen_predictive():
    """S=8 posterior samples of a 2-layer RBF DGP scored on N_t=100 points."""
    rng = np.random.default_rng(20)
    p = make_params(["RBF", "RBF"], [30, 30], [5, 1], 4, 1, False, "gaussian", 20, 0.3, rng)
    Xt = rng.standard_normal((100, 4))
    Yt = rng.standard_normal((100, 1))
    S = 8
    Ws = [[rng.standard_normal(w.shape) for w in p.W] for _ in range(S)]
    lps, ses = [], []
    for s in range(S):
        p.W = [w.copy() for w in Ws[s]]
        lp, se = O.eval_log_likelihood_and_se(p, Xt, Yt)
        lps.append(lp)
        ses.append(se)
    out = {"Xt": Xt, "Yt": Yt, "y_std": np.array(1.7)}
    pack_params(p, out)
    for s in range(S):
        for l in range(p.L):
            out[f"Ws{s}_{l}"] = Ws[s][l]
    out["logp"], out["se"] = np.stack(lps), np.stack(ses)
    ll, rmse = O.predictive_summary(out["logp"], out["se"], y_std=1.7)
    out["LL"], out["RMSE"] = np.array(ll), np.array(rmse)
    np.savez_compressed(os.path.join(OUT, "predictive.npz"), **out)


def gen_precond():
    """RMSprop masses (models/dgp.py:252-296) from K=4 minibatch gradients."""
    rng = np.random.default_rng(30)
    p = make_params(["RBF", "RBF"], [16, 24], [3, 1], 2, 1, False, "gaussian", 30, 0.1, rng)
    K, B, N = 4, 16, 200
    Xs = rng.standard_normal((K, B, 2))
    Ys = rng.standard_normal((K, B, 1))
    grads = [O.grad_W(p, Xs[k], Ys[k], N) for k in range(K)]
    out = {"Xs": Xs, "Ys": Ys, "N": np.array(N)}
    pack_params(p, out)
    for centered in (False, True):
        M = O.precond_masses(grads, centered=centered)
        out["M_centered" if centered else "M"] = np.array(M)
    np.savez_compressed(os.path.join(OUT, "precond.npz"), **out)


if __name__ == "__main__":
    for k, v in CASES.items():
        gen_case(k, v)
    gen_config1_sgld()
    gen_predictive()
    gen_precond()
    print("written:", sorted(f for f in os.listdir(OUT) if f.endswith(".npz")))
