"""CPU oracle of the DGP-RF SGHMC/SGLD hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; the
product (dgp-rf-mcmc_amd/) never does, and fails loudly when its HIP library is missing.

This is a numpy restatement of the reference algorithm (shixinxing/DGP-RF-MCMC, TensorFlow 2
eager).  Every function names the reference lines it follows.  It runs in float64 by default
(the parity reference) or float32 (`dtype=np.float32`, the op-for-op "reference-algorithm CPU
proxy" timed by bench.py, since TensorFlow itself is not installed here or on the GPU box).

PARITY STATUS: **parity unpinned against the reference's own outputs.**  The reference ships no
tests, fixtures or seeds, TensorFlow is not importable in this image (ModuleNotFoundError, not a
permission denial), and TF's unseeded global RNG cannot be replayed.  What pins this restatement:
  * the reference's own printed known answers: the cyclical schedule values printed by the
    notebooks (experiments/train_regression_*.ipynb "lr = ..."), the initial kernel
    hyper-parameters (train_regression_EM_mcycle.ipynb cell 5, train_regression_demo_sin.ipynb
    cell 5) — tests/test_oracle_golden.py;
  * the analytic backward pass against torch-CPU autograd of the same forward (a second,
    independent differentiation, like the reference's GradientTape) and finite differences —
    tests/test_oracle_autograd.py;
  * Philox4x32-10 against the published Random123 known-answer vectors — tests/test_oracle_rng.py.
"""
import numpy as np

LOG_2PI = np.log(2.0 * np.pi)


# ----------------------------------------------------------------------------- construction
def layer_widths(d_in, n_gp, input_cat):
    """Per-layer RF input widths: [d_in, n_gp[:-1]] (+ d_in if input_cat) — models/dgp.py:76-79."""
    if not input_cat:
        return [d_in] + list(n_gp[:-1])
    return [d_in] + [g + d_in for g in n_gp[:-1]]


def phi_width(kind, R):
    """GPLayer input width: 2R for RBF, R for ARC — models/dgp.py:103,107."""
    return 2 * R if kind == "RBF" else R


def init_log_inv_ls(d):
    """ARD init: length_scale = sqrt(d) broadcast to [d] (is_ard=True) — kernels/RBF.py:16-24,40."""
    return np.full(d, -0.5 * np.log(d))


class Params:
    """All state the reference keeps in tf.Variables of one DGP_RF (models/dgp.py:9-115)."""

    def __init__(self, d_in, d_out, n_rf, n_gp, kinds, likelihood="gaussian", input_cat=False,
                 z=None, W=None, log_amp=None, log_inv_ls=None, mean=None, lik_log_var=None,
                 rng=None, dtype=np.float64):
        L = len(n_rf)
        assert len(n_gp) == L and len(kinds) == L, "Error in #hidden GP layers!"  # dgp.py:38,43
        self.d_in, self.d_out, self.L = d_in, d_out, L
        self.n_rf, self.n_gp, self.kinds = list(n_rf), list(n_gp), list(kinds)
        self.likelihood, self.input_cat, self.dtype = likelihood, input_cat, dtype
        self.d = layer_widths(d_in, n_gp, input_cat)
        self.P = [phi_width(k, r) for k, r in zip(kinds, n_rf)]
        rng = rng if rng is not None else np.random.default_rng(0)
        c = lambda a: np.asarray(a, dtype=dtype)
        self.z = [c(z[l]) if z is not None else c(rng.standard_normal((self.d[l], n_rf[l])))
                  for l in range(L)]
        self.W = [c(W[l]) if W is not None else c(rng.standard_normal((self.P[l], n_gp[l])))
                  for l in range(L)]
        self.log_amp = [c(0.0 if log_amp is None else log_amp[l]) for l in range(L)]
        self.log_inv_ls = [c(init_log_inv_ls(self.d[l]) if log_inv_ls is None else log_inv_ls[l])
                           for l in range(L)]
        self.mean = [c(np.zeros(self.d[l]) if mean is None else mean[l]) for l in range(L)]
        self.lik_log_var = c(np.log(0.1) if lik_log_var is None else lik_log_var)  # gaussian.py:7,12


# ----------------------------------------------------------------------------- forward
def omega(p, l):
    """Omega = exp(log_inv_ls)[:, None] * z + mean — layers/rf_layers.py:34-38, kernels/RBF.py:51-53."""
    return np.exp(p.log_inv_ls[l])[:, None] * p.z[l] + p.mean[l][:, None]


def amp_scale(p, l):
    """c_l: amplitude/sqrt(R) (RBF, rf_layers.py:44) or sqrt(2)*amplitude/sqrt(R) (ARC, :90)."""
    amp = np.exp(p.log_amp[l])
    R = p.dtype(p.n_rf[l]) if p.dtype is np.float32 else float(p.n_rf[l])
    if p.kinds[l] == "RBF":
        return amp / np.sqrt(R)
    return np.sqrt(p.dtype(2.0)) * amp / np.sqrt(R)


def rf_features(p, l, X):
    """RBFLayer/ARCLayer.__call__ — layers/rf_layers.py:29-45 (cos block then sin block), :75-91."""
    A = X @ omega(p, l)
    c = amp_scale(p, l)
    if p.kinds[l] == "RBF":
        return A, c * np.concatenate([np.cos(A), np.sin(A)], axis=-1)
    return A, c * np.maximum(A, 0)


def forward(p, X, keep=False):
    """BNN_from_list(_input_cat).__call__ — utils.py:10-16 / 32-44 ([F | X] concat, F first).

    Returns F_L, or (F_L, per-layer cache) with keep=True.
    """
    X = np.asarray(X, dtype=p.dtype)
    F = X
    cache = []
    for l in range(p.L):
        Xin = F if (l == 0 or not p.input_cat) else np.concatenate([F, X], axis=-1)
        A, Phi = rf_features(p, l, Xin)
        F = Phi @ p.W[l]                                    # layers/GP_weight_layers.py:13
        cache.append((Xin, A, Phi, F))
    return (F, cache) if keep else F


def log_prob(p, F, Y):
    """Gaussian.log_prob (likelihoods/gaussian.py:18-25, utils.py:46-47) or Softmax.log_prob
    (likelihoods/softmax.py:8-15, -sparse_softmax_xent with int32(Y[:,0]))."""
    if p.likelihood == "gaussian":
        var = np.exp(p.lik_log_var)
        return np.sum(-0.5 * (LOG_2PI + np.log(var) + (Y - F) ** 2 / var), axis=-1)
    lab = np.asarray(Y)[:, 0].astype(np.int32)
    mx = F.max(axis=-1, keepdims=True)
    lse = mx[:, 0] + np.log(np.exp(F - mx).sum(axis=-1))
    return F[np.arange(F.shape[0]), lab] - lse


def prior_W(p):
    """sum_l sum log N(W_l; 0, 1) — models/dgp.py:129-136."""
    return sum(np.sum(-0.5 * (LOG_2PI + 0.0 + w ** 2)) for w in p.W)


def U(p, X, Y, N):
    """Minibatch potential, full_bayesian=False — models/dgp.py:161-182."""
    B = X.shape[0]
    return -(prior_W(p) / N + np.sum(log_prob(p, forward(p, X), Y)) / B)


# ----------------------------------------------------------------------------- backward
def dlogp_dF(p, F, Y):
    """d log p / dF per row — derivative of likelihoods/gaussian.py:24 / softmax.py:15."""
    if p.likelihood == "gaussian":
        return (Y - F) / np.exp(p.lik_log_var)
    lab = np.asarray(Y)[:, 0].astype(np.int32)
    mx = F.max(axis=-1, keepdims=True)
    sm = np.exp(F - mx)
    sm /= sm.sum(axis=-1, keepdims=True)
    oh = np.zeros_like(F)
    oh[np.arange(F.shape[0]), lab] = 1.0
    return oh - sm


def grad_W(p, X, Y, N):
    """dU/dW_l for every layer: the analytic form of tape.gradient (models/dgp.py:194-198).

    dF_L = -(1/B) dlogp/dF; for l = L..1: gW_l = Phi_l^T dF_l + W_l/N; dPhi = dF W^T;
    RBF: dA = c(-sin A * dPhi_cos + cos A * dPhi_sin); ARC: dA = c 1[A>0] dPhi;
    dX = dA Omega^T; dF_{l-1} = dX[:, :g_{l-1}].
    """
    X = np.asarray(X, dtype=p.dtype)
    B = X.shape[0]
    F, cache = forward(p, X, keep=True)
    dF = -dlogp_dF(p, F, Y) / B
    grads = [None] * p.L
    for l in reversed(range(p.L)):
        Xin, A, Phi, _ = cache[l]
        grads[l] = Phi.T @ dF + p.W[l] / N
        if l == 0:
            break
        dPhi = dF @ p.W[l].T
        c = amp_scale(p, l)
        R = p.n_rf[l]
        if p.kinds[l] == "RBF":
            dA = c * (-np.sin(A) * dPhi[:, :R] + np.cos(A) * dPhi[:, R:])
        else:
            dA = c * (A > 0) * dPhi
        dX = dA @ omega(p, l).T
        dF = dX[:, :p.n_gp[l - 1]]
    return grads


# ----------------------------------------------------------------------------- full Bayes
class Trainable:
    """Which hyper-parameters are tf.Variables with trainable=True in the reference:
    kernel log_amplitude / log_inv_length_scale (kernel_trainable, models/dgp.py:58-73,
    kernels/RBF.py:39-41), the layer means (set_nonzero_mean, layers/rf_layers.py:23-26) and the
    Gaussian lik_log_var (likelihoods/gaussian.py:12); `ard[l]` False = one scalar length scale
    for layer l (all d slots equal, gradient summed over them)."""

    def __init__(self, kernel=True, lik=True, mean=False, ard=None):
        self.kernel, self.lik, self.mean, self.ard = kernel, lik, mean, ard


def U_full(p, X, Y, N, tr):
    """Minibatch potential, full_bayesian=True — models/dgp.py:175-181: the N(0,1) prior over every
    trainable variable (W, kernel hyper-parameters, means, lik_log_var) divided by N."""
    B = X.shape[0]
    lg = lambda v: np.sum(-0.5 * (LOG_2PI + np.asarray(v) ** 2))
    pri = prior_W(p)
    for l in range(p.L):
        if tr.kernel:
            pri += lg(p.log_amp[l])
            ard = tr.ard is None or tr.ard[l]
            pri += lg(p.log_inv_ls[l] if ard else p.log_inv_ls[l][:1])
        if tr.mean:
            pri += lg(p.mean[l])
    if tr.lik and p.likelihood == "gaussian":
        pri += lg(p.lik_log_var)
    return -(pri / N + np.sum(log_prob(p, forward(p, X), Y)) / B)


def grad_full(p, X, Y, N, tr):
    """dU/d(every trainable variable), full_bayesian=True — the analytic form of tape.gradient
    over self.trainable_variables (models/dgp.py:199-204).  Per layer (all layers):
      gW = Phi^T dF + W/N,  dPhi = dF W^T,  g_log_amp = sum(dPhi * Phi) + log_amp/N
      dA as in grad_W,  G = X_l^T dA  (dU/dOmega),  Omega = exp(lis) z + mean:
      g_lis[k] = exp(lis[k]) sum_f G[k,f] z[k,f] + lis[k]/N   (scalar lis: summed over k)
      g_mean[k] = sum_f G[k,f] + mean[k]/N
    and g_lik_log_var = (1/B) sum_b sum_o (1 - (y-F)^2/var)/2 + lik_log_var/N (Gaussian).
    Returns a dict of per-layer lists (+ 'lik_log_var'); entries of non-trainable groups are None.
    """
    X = np.asarray(X, dtype=p.dtype)
    B = X.shape[0]
    F, cache = forward(p, X, keep=True)
    dF = -dlogp_dF(p, F, Y) / B
    out = {"W": [None] * p.L, "log_amp": [None] * p.L, "log_inv_ls": [None] * p.L,
           "mean": [None] * p.L, "lik_log_var": None}
    for l in reversed(range(p.L)):
        Xin, A, Phi, _ = cache[l]
        out["W"][l] = Phi.T @ dF + p.W[l] / N
        dPhi = dF @ p.W[l].T
        c = amp_scale(p, l)
        R = p.n_rf[l]
        if tr.kernel:
            out["log_amp"][l] = np.sum(dPhi * Phi) + p.log_amp[l] / N
        if p.kinds[l] == "RBF":
            dA = c * (-np.sin(A) * dPhi[:, :R] + np.cos(A) * dPhi[:, R:])
        else:
            dA = c * (A > 0) * dPhi
        G = Xin.T @ dA
        if tr.kernel:
            g = np.exp(p.log_inv_ls[l]) * np.sum(G * p.z[l], axis=1)
            ard = tr.ard is None or tr.ard[l]
            if ard:
                out["log_inv_ls"][l] = g + p.log_inv_ls[l] / N
            else:
                out["log_inv_ls"][l] = np.sum(g) + p.log_inv_ls[l][0] / N
        if tr.mean:
            out["mean"][l] = np.sum(G, axis=1) + p.mean[l] / N
        if l > 0:
            dF = (dA @ omega(p, l).T)[:, :p.n_gp[l - 1]]
    if tr.lik and p.likelihood == "gaussian":
        var = np.exp(p.lik_log_var)
        out["lik_log_var"] = np.sum(0.5 * (1.0 - (Y - F) ** 2 / var)) / B + p.lik_log_var / N
    return out


# ----------------------------------------------------------------------------- update
def sghmc_update(W, m, g, lr, N, beta, T, M, xi, xi_resample=None):
    """One SGHMC/SGLD update of one parameter tensor — models/dgp.py:206-216.

    h = sqrt(lr/N); [m <- xi_resample (ignores M)]; m <- beta m - h N g + sqrt(2(1-beta) T M) xi;
    W <- W + h m / M.  Returns (W_new, m_new).
    """
    h = np.sqrt(lr / N)
    if xi_resample is not None:
        m = xi_resample
    m_new = beta * m - h * N * g
    m_new = m_new + np.sqrt(2.0 * (1.0 - beta) * T * M) * xi
    return W + h * (1.0 / M) * m_new, m_new


def sgmcmc_step(p, m_list, X, Y, N, lr, beta, T, M_list, xi_list, xi_resample_list=None):
    """DGP_RF.sgmcmc_update with injected noise (models/dgp.py:184-216); updates p.W in place."""
    g = grad_W(p, X, Y, N)
    out_m = []
    for l in range(p.L):
        xr = None if xi_resample_list is None else xi_resample_list[l]
        p.W[l], m_new = sghmc_update(p.W[l], m_list[l], g[l], lr, N, beta, T, M_list[l],
                                     xi_list[l], xr)
        out_m.append(m_new)
    return out_m


def full_groups(p, tr):
    """The trainable variables of full_bayesian=True in a fixed order, as (name, layer) keys:
    per layer W, log_amp, log_inv_ls, mean (when trainable), then lik_log_var."""
    keys = []
    for l in range(p.L):
        keys.append(("W", l))
        if tr.kernel:
            keys += [("log_amp", l), ("log_inv_ls", l)]
        if tr.mean:
            keys.append(("mean", l))
    if tr.lik and p.likelihood == "gaussian":
        keys.append(("lik_log_var", None))
    return keys


def get_var(p, key, tr):
    name, l = key
    if name == "lik_log_var":
        return np.asarray(p.lik_log_var)
    v = getattr(p, name)[l]
    if name == "log_inv_ls" and tr.ard is not None and not tr.ard[l]:
        return np.asarray(v[0])
    return np.asarray(v)


def set_var(p, key, tr, value):
    name, l = key
    if name == "lik_log_var":
        p.lik_log_var = np.asarray(value, dtype=p.dtype)
        return
    if name == "log_inv_ls" and tr.ard is not None and not tr.ard[l]:
        p.log_inv_ls[l] = np.full(p.d[l], value, dtype=p.dtype)
        return
    getattr(p, name)[l] = np.asarray(value, dtype=p.dtype)


def sgmcmc_step_full(p, mom, X, Y, N, lr, beta, T, M, xi, tr, xi_resample=None):
    """DGP_RF.sgmcmc_update(full_bayesian=True) with injected noise (models/dgp.py:199-216): every
    trainable variable takes the same SGHMC update with its own momentum `mom[key]`, mass
    `M[key]` and noise `xi[key]` (gradients all taken at the pre-update state)."""
    g = grad_full(p, X, Y, N, tr)
    new_mom = {}
    for key in full_groups(p, tr):
        name, l = key
        gk = g[name] if name == "lik_log_var" else g[name][l]
        xr = None if xi_resample is None else xi_resample[key]
        v, m = sghmc_update(get_var(p, key, tr), mom[key], gk, lr, N, beta, T, M[key], xi[key], xr)
        set_var(p, key, tr, v)
        new_mom[key] = m
    return new_mom


# ----------------------------------------------------------------------------- preconditioner
def welford(mean, m2, g, k):
    """models/dgp.py:268-271."""
    delta = g - mean
    mean = mean + delta / k
    delta2 = g - mean
    return mean, m2 + delta * delta2


def mass_estimate(mean, m2, K, centered):
    """models/dgp.py:280-288 (DEFAULT_REGULARIZATION = 1e-7, :250)."""
    if centered:
        sq = np.mean(m2 / (K - 1))
    else:
        sq = np.mean(mean ** 2 + m2 / K)
    return np.sqrt(sq + 1.0e-7)


def precond_masses(grad_samples, centered=False):
    """RMSprop masses of models/dgp.py:252-296 from K gradient samples per parameter.

    grad_samples: list over K of lists over layers.  Returns M_l = mass_l / min_l mass_l.
    """
    K = len(grad_samples)
    L = len(grad_samples[0])
    masses = []
    for l in range(L):
        mean = np.zeros_like(grad_samples[0][l])
        m2 = np.zeros_like(grad_samples[0][l])
        for k in range(K):
            mean, m2 = welford(mean, m2, grad_samples[k][l], k + 1)
        masses.append(mass_estimate(mean, m2, K, centered))
    mmin = min(masses)
    return [m / mmin for m in masses]


# ----------------------------------------------------------------------------- schedule
def cyclical_step_rate(step_index, cycle_length, schedule="cosine", min_value=0.001,
                       dtype=np.float32):
    """utils.py:49-73 (float32 like the TF ops).  Returns (rate, is_end)."""
    if step_index <= 0:
        raise ValueError("Step index should be larger than zero!")
    frac = dtype((step_index - 1) % cycle_length) / dtype(cycle_length)
    if schedule == "cosine":
        rate = dtype(min_value) + dtype(1.0 - min_value) * dtype(0.5) * (
            np.cos(dtype(np.pi) * frac) + dtype(1.0))
    elif schedule == "glide":
        rate = dtype(min_value) + dtype(1.0 - min_value) * np.exp(-frac / (dtype(1.0) - frac))
    elif schedule == "flat":
        rate = dtype(1.0)
    else:
        raise NotImplementedError
    return dtype(rate), (step_index % cycle_length) == 0


# ----------------------------------------------------------------------------- predictive
def eval_log_likelihood_and_se(p, X, Y):
    """RegressionDGP.eval_log_likelihood_and_se — models/regression_model.py:33-50."""
    F = forward(p, X)
    return log_prob(p, F, Y), np.mean((Y - F) ** 2, axis=-1)


def predictive_summary(log_p, se, y_std=1.0):
    """experiments/utils_training.py:63-65,79-85: LL = mean_n[LSE_s(lp - log y_std) - log S],
    RMSE = sqrt(mean_{s,n}(se * y_std^2)).  log_p, se: [S, N]."""
    lp = np.asarray(log_p, dtype=np.float64) - np.log(y_std)
    S = lp.shape[0]
    mx = lp.max(axis=0)
    lse = mx + np.log(np.exp(lp - mx).sum(axis=0))
    ll = np.mean(lse - np.log(S))
    rmse = np.sqrt(np.mean(np.asarray(se, dtype=np.float64) * y_std ** 2))
    return ll, rmse


# ----------------------------------------------------------------------------- MCEM M-step
def q_function_and_grad(p, W_samples, X, Y, N, tr):
    """MCEM_Q_maximizer (experiments/utils_training.py:339-358, utils_training_demo.py:171-191):
    Q = (1/S) sum_s -U(W_s; full_bayesian=False, allow_gradient_from_W=False)
      = (1/S) sum_s (1/B) sum_b log p(y_b | x_b, W_s)        (no prior: dgp.py:169-174)
    and d(-Q)/d(hyper) for the watched Omega_hyperparams + Likelihood_hyperparams, which is the
    full-Bayes hyper-parameter gradient of grad_full without its prior term hyper/N.
    W_samples: list over S of per-layer W lists.  Returns (Q, dict like grad_full minus 'W');
    p.W is left at the last sample (the reference's assign_W leaves it there too)."""
    X = np.asarray(X, dtype=p.dtype)
    B = X.shape[0]
    Q = 0.0
    acc = None
    for Ws in W_samples:
        p.W = [np.asarray(w, dtype=p.dtype).copy() for w in Ws]
        Q += np.sum(log_prob(p, forward(p, X), Y)) / B
        g = grad_full(p, X, Y, N, tr)
        g.pop("W")
        if acc is None:
            acc = g
            continue
        for k in ("log_amp", "log_inv_ls", "mean"):
            acc[k] = [a if a is None else a + b for a, b in zip(acc[k], g[k])]
        if acc["lik_log_var"] is not None:
            acc["lik_log_var"] = acc["lik_log_var"] + g["lik_log_var"]
    S = len(W_samples)
    out = {"log_amp": [None] * p.L, "log_inv_ls": [None] * p.L, "mean": [None] * p.L,
           "lik_log_var": None}
    for l in range(p.L):
        if acc["log_amp"][l] is not None:
            out["log_amp"][l] = acc["log_amp"][l] / S - p.log_amp[l] / N
        if acc["log_inv_ls"][l] is not None:
            ard = tr.ard is None or tr.ard[l]
            lis = p.log_inv_ls[l] if ard else p.log_inv_ls[l][0]
            out["log_inv_ls"][l] = acc["log_inv_ls"][l] / S - lis / N
        if acc["mean"][l] is not None:
            out["mean"][l] = acc["mean"][l] / S - p.mean[l] / N
    if acc["lik_log_var"] is not None:
        out["lik_log_var"] = acc["lik_log_var"] / S - p.lik_log_var / N
    return Q / S, out


def adam_update(var, g, m, v, t, lr=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-7):
    """One tf.keras.optimizers.Adam step (the optimizer the reference's MCEM notebooks pass to
    MCEM_Q_maximizer, experiments/train_classification.ipynb cell 'optimizer = optimizers.Adam',
    defaults of TF2 Keras Adam):  t = iteration (from 1),
      lr_t = lr sqrt(1 - beta_2^t) / (1 - beta_1^t),  m <- beta_1 m + (1 - beta_1) g,
      v <- beta_2 v + (1 - beta_2) g^2,  var <- var - lr_t m / (sqrt(v) + epsilon).
    Returns (var, m, v)."""
    lr_t = lr * np.sqrt(1.0 - beta_2 ** t) / (1.0 - beta_1 ** t)
    m = beta_1 * m + (1.0 - beta_1) * g
    v = beta_2 * v + (1.0 - beta_2) * g * g
    return var - lr_t * m / (np.sqrt(v) + epsilon), m, v
