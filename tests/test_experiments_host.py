"""Host-side pieces of the experiments/ drivers (no GPU): the MCEM oracle (Q and its hyper-parameter
gradient) against finite differences, the Keras-Adam restatement, the UCI split / normalisation of
experiments/datasets.py, the tf.data stand-in, and the sampler's schedule bookkeeping
(experiments/utils_training.py:41-70) driven through a recording stand-in model."""
import numpy as np
import pytest
import torch

from oracle import dgp_oracle as O


# ----------------------------------------------------------------------------- MCEM oracle
@pytest.mark.parametrize("kinds,n_rf,n_gp,d_in,d_out,cat,lik,mean", [
    (["RBF"], [15], [1], 2, 1, False, "gaussian", False),
    (["RBF", "ARC"], [12, 10], [3, 2], 3, 2, True, "gaussian", True),
    (["ARC", "RBF"], [9, 11], [3, 4], 2, 4, False, "softmax", False),
])
def test_q_grad_matches_finite_differences(kinds, n_rf, n_gp, d_in, d_out, cat, lik, mean):
    """d(-Q)/d(hyper) of MCEM_Q_maximizer (utils_training.py:339-358) by central differences of
    Q(hyper) over S = 3 W samples; no prior term (U with allow_gradient_from_W=False)."""
    rng = np.random.default_rng(11)
    p = O.Params(d_in, d_out, n_rf, n_gp, kinds, lik, cat, rng=rng,
                 log_amp=[0.1 * (l + 1) for l in range(len(kinds))], lik_log_var=np.log(0.2),
                 mean=[0.1 * rng.standard_normal(w) for w in O.layer_widths(d_in, n_gp, cat)])
    tr = O.Trainable(kernel=True, lik=True, mean=mean)
    B, N = 17, 300
    X = rng.standard_normal((B, d_in))
    Y = rng.standard_normal((B, d_out)) if lik == "gaussian" else \
        rng.integers(0, d_out, (B, 1)).astype(float)
    Ws = [[rng.standard_normal(w.shape) for w in p.W] for _ in range(3)]
    Q, g = O.q_function_and_grad(p, Ws, X, Y, N, tr)

    def Qof():
        return O.q_function_and_grad(p, Ws, X, Y, N, tr)[0]
    eps = 1e-6
    for key in O.full_groups(p, tr):
        if key[0] == "W":
            continue
        name, l = key
        v0 = np.array(O.get_var(p, key, tr), dtype=np.float64)
        num = np.zeros_like(v0)
        for idx in np.ndindex(v0.shape if v0.shape else (1,)):
            v = v0.copy().reshape(-1) if v0.shape else v0.reshape(1).copy()
            j = np.ravel_multi_index(idx, v0.shape) if v0.shape else 0
            v[j] += eps
            O.set_var(p, key, tr, v.reshape(v0.shape))
            qp = Qof()
            v[j] -= 2 * eps
            O.set_var(p, key, tr, v.reshape(v0.shape))
            qm = Qof()
            O.set_var(p, key, tr, v0)
            num.reshape(-1)[j] = -(qp - qm) / (2 * eps)
        ana = g[name] if name == "lik_log_var" else g[name][l]
        np.testing.assert_allclose(ana, num, rtol=2e-5, atol=1e-7, err_msg=str(key))
    assert np.isfinite(Q)


def test_adam_matches_keras_rule():
    """experiments/optimizers.Adam (in place on tensors) vs the numpy restatement of Keras Adam."""
    from experiments.optimizers import Adam
    rng = np.random.default_rng(3)
    v1 = torch.tensor(rng.standard_normal(5), dtype=torch.float32)
    v2 = torch.tensor(0.3, dtype=torch.float32)
    opt = Adam(learning_rate=0.05)
    r1, r2 = v1.double().numpy().copy(), np.float64(0.3)
    m1 = s1 = np.zeros(5)
    m2 = s2 = 0.0
    for t in range(1, 5):
        g1 = rng.standard_normal(5)
        g2 = rng.standard_normal()
        opt.apply_gradients([(torch.tensor(g1, dtype=torch.float32), v1),
                             (torch.tensor(g2, dtype=torch.float32), v2)])
        r1, m1, s1 = O.adam_update(r1, g1, m1, s1, t, lr=0.05)
        r2, m2, s2 = O.adam_update(r2, g2, m2, s2, t, lr=0.05)
    np.testing.assert_allclose(v1.numpy(), r1, rtol=1e-5, atol=1e-6)
    assert abs(float(v2) - r2) < 1e-6
    assert opt.iterations == 4


# ----------------------------------------------------------------------------- datasets
def _write_csv(tmp_path, name, N, D, seed=0):
    rng = np.random.default_rng(seed)
    data = np.concatenate([rng.standard_normal((N, D)) * 3 + 1,
                           rng.standard_normal((N, 1)) * 5 + 2], axis=1)
    np.savetxt(tmp_path / f"{name}.csv", data, delimiter=",")
    return data


def test_uci_split_and_normalise(tmp_path):
    """experiments/datasets.py:47-87: legacy-seeded 90/10 split (bit-exact index work), X scaled by
    the train std + 1e-6, Y centred only; utils_dataset.download_UCI_data_info shapes."""
    from experiments import utils_dataset as U
    data = _write_csv(tmp_path, "boston", 506, 13)
    X, Y, Xs, Ys, X_mean, Y_mean, Y_std = U.download_UCI_data_info("boston",
                                                                    data_path=str(tmp_path) + "/")
    ind = np.arange(506)
    np.random.seed(0)
    np.random.shuffle(ind)
    n = int(506 * 0.9)
    Xtr, Ytr = data[ind[:n], :-1], data[ind[:n], -1:]
    m, s = Xtr.mean(0), Xtr.std(0) + 1e-6
    assert X.shape == (n, 13) and Xs.shape == (506 - n, 13) and Y.shape == (n, 1)
    np.testing.assert_allclose(X, ((Xtr - m) / s).astype(np.float32), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(Xs, ((data[ind[n:], :-1] - m) / s).astype(np.float32),
                               rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(Y, (Ytr - Ytr.mean()).astype(np.float32), rtol=1e-5, atol=1e-4)
    assert np.allclose(Y_mean, Ytr.mean()) and Y_std.tolist() == [1.0]
    with pytest.raises(FileNotFoundError):
        U.download_UCI_data_info("concrete", data_path=str(tmp_path) + "/")


def test_device_dataset_pipeline():
    """tf.data stand-in: shuffle each pass, batch with / without drop_remainder, repeat, map."""
    from experiments.utils_dataset import DeviceDataset
    cpu = torch.device("cpu")
    X = torch.arange(23, dtype=torch.float32)[:, None].repeat(1, 2)
    Y = torch.arange(23, dtype=torch.float32)
    ds = DeviceDataset(X, Y, dev=cpu).shuffle(23, seed=5).batch(5, drop_remainder=True)
    assert len(ds) == 4
    p1 = [b for b in ds]
    p2 = [b for b in ds]
    assert all(x.shape == (5, 2) and y.shape == (5, 1) for x, y in p1)
    r1 = torch.cat([y for _, y in p1]).reshape(-1)
    r2 = torch.cat([y for _, y in p2]).reshape(-1)
    assert len(set(r1.tolist())) == 20 and not torch.equal(r1, r2)  # reshuffled each pass
    for x, y in p1:
        assert torch.equal(x[:, 0], y[:, 0])  # rows stay paired
    full = DeviceDataset(X, Y, dev=cpu).batch(5)
    assert [len(y) for _, y in full] == [5, 5, 5, 5, 3]
    assert torch.equal(torch.cat([y for _, y in full]).reshape(-1), Y)  # unshuffled order
    it = iter(DeviceDataset(X, Y, dev=cpu).batch(10, drop_remainder=True).repeat())
    assert [next(it)[1][0, 0].item() for _ in range(5)] == [0, 10, 0, 10, 0]
    dm = full.map(lambda a, b: (a * 2, b))
    assert torch.equal(next(iter(dm))[0], X[:5] * 2)


# ----------------------------------------------------------------------------- driver schedule
class _Recorder:
    """Stand-in model recording the sgmcmc_update calls of the per-batch driver path."""

    def __init__(self):
        self.calls = []
        self.precond = 0
        self.n_hidden_layers = 1

    def precond_update(self, ds, data_size, **kw):
        self.precond += 1

    def sgmcmc_update(self, X, Y, data_size, lr, momentum_decay, full_bayesian,
                      resample_moments, temperature):
        self.calls.append((float(lr), float(temperature), bool(resample_moments)))


@pytest.mark.parametrize("resample", [False, True])
def test_driver_schedule_matches_reference_loop(resample):
    """experiments/utils_training.py:41-70: burn-in at lr_0 / T = 0, then lr_0 rate^2 / T = 1 with
    cycle-head momentum resampling, a sample at every cycle end."""
    from experiments.utils_training import _run_epochs
    from utils import cyclical_step_rate
    batches = [(np.zeros((2, 1)), np.zeros((2, 1)))] * 3  # 3 iterations per epoch
    rec = _Recorder()
    samples = []
    _run_epochs(rec, batches, batches, 6, 2, 0.05, 0.9, False, 'identity', None, None, resample,
                total_epochs=9, start_sampling_epoch=3, epochs_per_cycle=2,
                on_sample=lambda e, lr: samples.append((e, lr)))
    assert rec.precond == 9 and len(rec.calls) == 27
    assert rec.calls[:9] == [(0.05, 0.0, False)] * 9
    ref = []
    for si in range(1, 19):
        rate, _ = cyclical_step_rate(si, 6, schedule='cosine', min_value=0.)
        ref.append((float(np.float32(0.05) * rate ** 2), 1.0, resample and si % 6 == 1))
    for got, exp in zip(rec.calls[9:], ref):
        assert got[1:] == exp[1:] and abs(got[0] - exp[0]) < 1e-9
    assert [e for e, _ in samples] == [4, 6, 8]
