"""experiments/ drivers on the HIP path: the MCEM M-step (device Q gradient + Adam) against the
oracle, and the graph-per-epoch sampling driver against per-step replays.

Tolerances (fp32 device vs float64 oracle): Q 2e-5 of its scale; d(-Q)/d(hyper) 5e-4 of each
group's scale (sums over every row and feature, like the full-Bayes gradients); one Adam step
1e-5 absolute on the hyper-parameters; driver vs manual graph replays bit-exact.
"""
import numpy as np
import pytest
import torch

from oracle import dgp_oracle as O
from test_gpu_full_bayes import close, group_err, hyper_of, trainable  # noqa: F401
from test_gpu_parity import cpu, dev, model_from_fixture, oracle_params  # noqa: F401

pytestmark = pytest.mark.gpu


def _w_samples(g, S, seed):
    rng = np.random.default_rng(seed)
    return [[g[f"W{l}"] + 0.3 * rng.standard_normal(g[f"W{l}"].shape)
             for l in range(len(g["kinds"]))] for _ in range(S)]


@pytest.mark.parametrize("name", ["rbf2_gauss", "arc_rbf_softmax_cat", "mixed5"])
def test_q_and_hyper_grads(dev, golden, name):
    """MCEM_Q_maximizer's Q and d(-Q)/d(Omega_hyperparams + Likelihood_hyperparams)
    (experiments/utils_training.py:339-358) over S = 3 W samples vs the oracle."""
    g = golden(name)
    m = model_from_fixture(g)
    eng = m._engine
    N_ = int(g["dims"][5])
    Ws = _w_samples(g, 3, 5)
    Q, grads = m.Q_and_hyper_grads(Ws, g["X"], g["Y"], N_)
    p = oracle_params(g)
    Qr, ref = O.q_function_and_grad(p, Ws, g["X"], g["Y"], N_, trainable(g, eng))
    assert abs(float(Q) - Qr) < 2e-5 * max(1.0, abs(Qr))
    # the model holds the last sample afterwards, like the reference's assign_W loop
    for l in range(m.n_hidden_layers):
        assert np.allclose(cpu(m.W_mcmc[l]), Ws[-1][l], atol=1e-6)
    vars_ = m.hyper_variables()
    assert len(grads) == len(vars_)
    L = m.n_hidden_layers
    # hyper_variables order: per layer log_amp, log_inv_ls, mean; then lik_log_var
    k = 0
    amp_dev, amp_ref = [], []
    for l in range(L):
        amp_dev.append(float(grads[k])); amp_ref.append(float(ref["log_amp"][l]))
        assert group_err(cpu(grads[k + 1]), ref["log_inv_ls"][l]) < 5e-4, (name, "lis", l)
        assert group_err(cpu(grads[k + 2]).reshape(-1), ref["mean"][l]) < 5e-4, (name, "mean", l)
        k += 3
    assert group_err(amp_dev, amp_ref) < 5e-4
    if ref["lik_log_var"] is not None:
        assert abs(float(grads[k]) - float(ref["lik_log_var"])) < \
            5e-4 * (abs(float(ref["lik_log_var"])) + 1.0)
        k += 1
    assert k == len(grads)


def test_mcem_maximizer_adam_step(dev, golden):
    """One M step: maximizer(W_samples, X, Y) applies Keras-rule Adam to the hyper-parameters on
    the device; Omega is rebuilt from them by the next call (forward matches the oracle)."""
    from experiments.optimizers import Adam
    from experiments.utils_training import MCEM_Q_maximizer
    g = golden("rbf2_gauss")
    m = model_from_fixture(g)
    eng = m._engine
    N_ = int(g["dims"][5])
    Ws = _w_samples(g, 2, 9)
    p = oracle_params(g)
    tr = trainable(g, eng)
    _, ref = O.q_function_and_grad(p, Ws, g["X"], g["Y"], N_, tr)
    opt = Adam(learning_rate=0.01)
    MCEM_Q_maximizer(m, N_, opt)(Ws, g["X"], g["Y"])
    for key in O.full_groups(p, tr):
        if key[0] == "W":
            continue
        name, l = key
        gk = ref[name] if name == "lik_log_var" else ref[name][l]
        v, _, _ = O.adam_update(O.get_var(p, key, tr), gk, 0.0, 0.0, 1, lr=0.01)
        O.set_var(p, key, tr, v)
    h = hyper_of(eng, eng.hyp_chain(0))
    for l in range(m.n_hidden_layers):
        assert close(h["log_amp"][l], p.log_amp[l], 1e-5)
        assert close(h["log_inv_ls"][l], p.log_inv_ls[l], 1e-5)
        assert close(h["mean"][l], p.mean[l], 1e-5)
    assert close(h["lik_log_var"], p.lik_log_var, 1e-5)
    F = cpu(m.BNN(g["X"]))
    p.W = [np.asarray(w, np.float64) for w in Ws[-1]]
    Fr = O.forward(p, g["X"])
    assert np.max(np.abs(F - Fr)) < 2e-5 * max(1.0, np.max(np.abs(Fr)))


def _small_regression(seed=0, n=600, n_test=97, d=3):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, d)).astype(np.float32)
    Y = np.sin(X @ rng.standard_normal((d, 1))).astype(np.float32)
    Xs = rng.standard_normal((n_test, d)).astype(np.float32)
    Ys = np.sin(Xs @ rng.standard_normal((d, 1))).astype(np.float32)
    return X, Y, Xs, Ys


def test_regression_train_graph_driver(dev):
    """regression_train (utils_training.py:11-88) with one hipGraph replay per epoch: the sample
    count of the cycle bookkeeping, finite [S, N_test] outputs, and the same final state as replaying
    the identical per-epoch graphs by hand (bit-exact)."""
    from dgprf import engine as E
    from experiments.utils_training import regression_train
    from likelihoods import Gaussian
    from models.regression_model import RegressionDGP
    data = _small_regression()
    finals = []
    for manual in (False, True):
        E.set_seed(4)
        m = RegressionDGP(3, 1, n_hidden_layers=2, n_rf=[64, 32], n_gp=[3, 1],
                          likelihood=Gaussian(variance=0.1))
        np.random.seed(1234)  # the train pipeline's shuffle seed comes from the legacy RNG
        if not manual:
            log_p, mse = regression_train(m, batch_size=100, lr_0=0.01, momentum_decay=0.9,
                                          full_bayesian=False, total_epochs=7,
                                          start_sampling_epoch=3, epochs_per_cycle=2,
                                          print_epoch_cycle=1000, data=data)
            assert tuple(log_p.shape) == (2, 97) and tuple(mse.shape) == (2, 97)
            assert torch.isfinite(log_p).all() and torch.isfinite(mse).all()
        else:
            from experiments.utils_dataset import load_arrays
            ds, _, _, _ = load_arrays(*data, batch_size=100)
            m.precond_update(None, 600, precond_type="identity")
            for _ in range(7):
                m.run_sgmcmc(ds.X, ds.Y, 600, 6, batch_size=100, lr=0.01, momentum_decay=0.9,
                             steps_per_graph=6, perm_seed=ds.seed, schedule='cyclical',
                             start_step=18, cycle_length=12)
        finals.append(m._engine.theta.clone())
    assert torch.equal(finals[0], finals[1])


def test_mcem_end_to_end(dev):
    """MCEM (utils_training.py:360-379) with MCEM_sampler_UCI on in-memory data: two EM steps move
    the hyper-parameters, the final fixed-hyper sampling returns [S, N_test] matrices."""
    from dgprf import engine as E
    from experiments.optimizers import Adam
    from experiments.utils_training import MCEM, MCEM_Q_maximizer, MCEM_sampler_UCI
    from likelihoods import Gaussian
    from models.regression_model import RegressionDGP
    data = _small_regression(1)
    E.set_seed(8)
    m = RegressionDGP(3, 1, n_hidden_layers=1, n_rf=50, n_gp=1, likelihood=Gaussian())
    kw = dict(batch_size=100, start_sampling_epoch=1, epochs_per_cycle=2, data=data)
    s_em = MCEM_sampler_UCI(m, **kw)
    s_fix = MCEM_sampler_UCI(m, **kw)
    h0 = m._engine.hyp.clone()
    log_p, mse = MCEM(s_em, MCEM_Q_maximizer(m, 600, Adam(0.05)), s_fix, 2, s_em.ds_train,
                      num_samples_EM=2, num_samples_fixing_hyper=3)
    assert tuple(log_p.shape) == (3, 97) and torch.isfinite(log_p).all()
    dh = (m._engine.hyp - h0).abs()
    assert float(dh.max()) > 0.01  # Adam moved the kernel / likelihood hyper-parameters


def test_eval_whole_test_set_equals_batches(dev):
    """eval_log_likelihood_and_se / eval_log_likelihood over an in-order DeviceDataset score every
    row in ONE forward (models.dgp.whole_dataset) instead of one per batch: the same rows in the
    same order as the batch loop (a plain list of the same batches, whose per-batch forward the
    parity tests pin to the oracle), to fp32 rounding of another kernel path; a drop_remainder set
    leaves out the same rows."""
    from dgprf import engine as E
    from experiments.utils_dataset import DeviceDataset, load_arrays
    from likelihoods import Gaussian, Softmax
    from models.classification_model import ClassificationDGP
    from models.regression_model import RegressionDGP
    X, Y, Xs, Ys = _small_regression(2, n_test=1003)
    E.set_seed(11)
    m = RegressionDGP(3, 1, n_hidden_layers=2, n_rf=[64, 32], n_gp=[3, 1],
                      likelihood=Gaussian(variance=0.1))
    _, ds_test, _, _ = load_arrays(X, Y, Xs, Ys, batch_size=100)
    lp, se = m.eval_log_likelihood_and_se(ds_test)
    lp_b, se_b = m.eval_log_likelihood_and_se([(x, y) for x, y in ds_test])
    assert lp.shape == (1003,) and se.shape == (1003,)
    scale = float(lp_b.abs().max())
    assert float((lp - lp_b).abs().max()) <= 2e-6 * scale
    assert float((se - se_b).abs().max()) <= 2e-6 * float(se_b.abs().max())
    dr = DeviceDataset(Xs, Ys).batch(100, drop_remainder=True)
    assert m.eval_log_likelihood_and_se(dr)[0].shape == (1000,)
    E.set_seed(12)
    c = ClassificationDGP(3, 4, n_hidden_layers=2, n_rf=[64, 32], n_gp=[5, 4],
                          likelihood=Softmax())
    Yc = (np.abs(Ys * 7).astype(np.int64) % 4).astype(np.float32)
    ds_c = DeviceDataset(Xs, Yc).batch(128)
    lc = c.eval_log_likelihood(ds_c)
    lc_b = c.eval_log_likelihood([(x, y) for x, y in ds_c])
    assert float((lc - lc_b).abs().max()) <= 2e-6 * float(lc_b.abs().max())
