"""HIP path (libdgprf.so via the C-ABI) against the CPU oracle and the golden fixtures.

Tolerances (fp32 device vs float64 oracle, stated per check): forward / log p rel 2e-5 of the
output scale, gradients 1e-4 of the gradient scale, one update 1e-5; minibatch indices and
graph-vs-eager replays bit-exact.
"""
import math

import numpy as np
import pytest
import torch

from oracle import dgp_oracle as O
from oracle import rng as R

pytestmark = pytest.mark.gpu

KIND = {0: "RBF", 1: "ARC"}


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b)) / (np.max(np.abs(b)) + 1e-30))


def cpu(t):
    return t.detach().float().cpu().numpy()


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    from dgprf import _native as N
    N.lib()
    return torch.device("cuda", 0)


def model_from_fixture(g):
    from likelihoods import Gaussian, Softmax
    from models.dgp import DGP_RF
    L = len(g["kinds"])
    d_in, d_out, cat, lik = (int(x) for x in g["dims"][:4])
    likelihood = Gaussian(variance=float(np.exp(g["lik_log_var"]))) if lik == 0 else Softmax()
    m = DGP_RF(d_in, d_out, n_hidden_layers=L, n_rf=[int(r) for r in g["n_rf"]],
               n_gp=[int(x) for x in g["n_gp"]], likelihood=likelihood,
               kernel_type_list=[KIND[int(k)] for k in g["kinds"]], input_cat=bool(cat),
               set_nonzero_mean=True)
    load_params(m, g)
    return m


def load_params(m, g, W_keys=None):
    with torch.no_grad():
        for l in range(m.n_hidden_layers):
            rf, gp = m.BNN.layers[2 * l], m.BNN.layers[2 * l + 1]
            rf.z.copy_(torch.as_tensor(g[f"z{l}"]))
            rf.kernel.log_amplitude.copy_(torch.as_tensor(g[f"log_amp{l}"]))
            rf.kernel.log_inv_length_scale.copy_(torch.as_tensor(g[f"log_inv_ls{l}"]))
            rf.mean.copy_(torch.as_tensor(g[f"mean{l}"])[:, None])
            gp.assign_W(g[(W_keys or "W{}").format(l)])
        if hasattr(m.likelihood, "lik_log_var"):
            m.likelihood.lik_log_var.copy_(torch.as_tensor(g["lik_log_var"]))


def oracle_params(g):
    L = len(g["kinds"])
    d_in, d_out, cat, lik = (int(x) for x in g["dims"][:4])
    return O.Params(d_in, d_out, list(g["n_rf"]), list(g["n_gp"]),
                    [KIND[int(k)] for k in g["kinds"]], "gaussian" if lik == 0 else "softmax",
                    bool(cat), z=[g[f"z{l}"] for l in range(L)], W=[g[f"W{l}"] for l in range(L)],
                    log_amp=[g[f"log_amp{l}"] for l in range(L)],
                    log_inv_ls=[g[f"log_inv_ls{l}"] for l in range(L)],
                    mean=[g[f"mean{l}"] for l in range(L)], lik_log_var=g["lik_log_var"])


def unpack(engine, flat, chain=0):
    pl = engine.layout
    out = []
    for l in range(engine.L):
        o, P, gg = pl.w_off[l], pl.P[l], pl.n_gp[l]
        out.append(cpu(flat[chain, o:o + P * gg]).reshape(P, gg))
    return out


def pack(engine, per_layer):
    t = torch.zeros(1, engine.layout.w_total, dtype=torch.float32)
    pl = engine.layout
    for l, a in enumerate(per_layer):
        o = pl.w_off[l]
        t[0, o:o + a.size] = torch.as_tensor(np.asarray(a, np.float32).reshape(-1))
    return t.to(engine.dev)


CASES = ["rbf2_gauss", "arc_rbf_softmax_cat", "mixed5", "wide_g"]


@pytest.mark.parametrize("n,P,g", [(1000, 2048, 30), (77, 8192, 16), (5, 6, 1), (33, 130, 17)])
def test_gp_layer_matmul(dev, n, P, g):
    """Stand-alone GPLayer.__call__ (layers/GP_weight_layers.py:11-15) on the MFMA tile kernel:
    ragged rows / outputs / K (P % 4 != 0 takes the scalar-load path) against float64 numpy."""
    from layers import GPLayer
    rng = np.random.default_rng(n + P)
    gp = GPLayer(P, g)
    W = rng.standard_normal((P, g)).astype(np.float32)
    gp.assign_W(W)
    X = (rng.standard_normal((n, P)) / np.sqrt(P)).astype(np.float32)
    F = cpu(gp(X))
    assert rel_err(F, X.astype(np.float64) @ W.astype(np.float64)) < 1e-5


# ----------------------------------------------------------------------------- RNG
def test_philox_normal_matches_oracle(dev):
    from dgprf import _native as N
    from dgprf import engine as E
    out = torch.empty(4099, dtype=torch.float32, device=dev)
    N.call("dgprf_philox_normal", E.ptr(out), out.numel(), 0xABCDEF1234, 77, R.PURPOSE_Z,
           E.stream())
    ref = R.philox_normal(4099, 0xABCDEF1234, 77, R.PURPOSE_Z)
    assert np.max(np.abs(cpu(out) - ref)) < 2e-5   # f32 log / sincospi vs float64


# ----------------------------------------------------------------------------- layers
@pytest.mark.parametrize("kind", ["RBF", "ARC"])
@pytest.mark.parametrize("n,d,R_", [(37, 3, 20), (1, 5, 100), (130, 40, 33)])
def test_rf_layer_standalone(dev, kind, n, d, R_):
    from kernels import ARCKernel, RBFKernel
    from layers import ARCLayer, GPLayer, RBFLayer
    k = (RBFKernel if kind == "RBF" else ARCKernel)(n_feature=d, is_ard=True)
    layer = (RBFLayer if kind == "RBF" else ARCLayer)(k, R_)
    rng = np.random.default_rng(n + d)
    with torch.no_grad():
        k.log_amplitude.fill_(0.3)
        k.log_inv_length_scale.copy_(torch.as_tensor(rng.normal(-0.5, 0.2, d)))
    X = rng.standard_normal((n, d))
    phi = cpu(layer(X))
    p = O.Params(d, 1, [R_], [1], [kind], z=[cpu(layer.z)], log_amp=[0.3],
                 log_inv_ls=[cpu(k.log_inv_length_scale)], mean=[np.zeros(d)])
    _, ref = O.rf_features(p, 0, X)
    assert phi.shape == ref.shape and rel_err(phi, ref) < 2e-5
    gp = GPLayer(phi.shape[1], 3)
    F = cpu(gp(torch.as_tensor(phi, device=dev)))
    assert rel_err(F, phi.astype(np.float64) @ cpu(gp.W)) < 2e-5


# ----------------------------------------------------------------------------- forward
@pytest.mark.parametrize("name", CASES)
def test_forward_and_likelihood(dev, golden, name):
    g = golden(name)
    m = model_from_fixture(g)
    L = m.n_hidden_layers
    F = cpu(m.BNN(g["X"]))
    assert rel_err(F, g[f"F{L - 1}"]) < 2e-5
    lp = cpu(m.log_likelihood(g["X"], g["Y"]))
    assert np.max(np.abs(lp - g["logp"])) < 2e-5 * max(1.0, np.max(np.abs(g["logp"])))
    U = float(m.U(g["X"], g["Y"], int(g["dims"][5])))
    assert abs(U - float(g["U"])) < 2e-5 * max(1.0, abs(float(g["U"])))
    assert abs(float(m.prior_W()) - float(g["prior_W"])) < 1e-5 * abs(float(g["prior_W"]))
    if int(g["dims"][3]) == 0:
        from models.regression_model import RegressionDGP
        lp2, se = RegressionDGP.eval_log_likelihood_and_se(m, [(g["X"][:10], g["Y"][:10]),
                                                               (g["X"][10:], g["Y"][10:])])
        assert np.max(np.abs(cpu(lp2) - g["logp"])) < 2e-5 * max(1.0, np.max(np.abs(g["logp"])))
        assert rel_err(cpu(se), g["se"]) < 5e-5
        if not int(g["dims"][2]):
            outs = RegressionDGP.feed_forward_all_layers(m, g["X"])
            for l in range(L):
                assert rel_err(cpu(outs[l]), g[f"F{l}"]) < 2e-5


# ----------------------------------------------------------------------------- backward
@pytest.mark.parametrize("name", CASES)
def test_potential_grad(dev, golden, name):
    g = golden(name)
    m = model_from_fixture(g)
    eng = m._engine
    G = unpack(eng, eng.grad(g["X"], g["Y"], int(g["dims"][5])))
    for l in range(m.n_hidden_layers):
        assert rel_err(G[l], g[f"g{l}"]) < 1e-4, (name, l)


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("resample", [False, True])
def test_sghmc_step_injected_noise(dev, golden, name, resample):
    g = golden(name)
    m = model_from_fixture(g)
    eng = m._engine
    L = m.n_hidden_layers
    lr, beta, T, N_ = g["step_scalars"]
    with torch.no_grad():
        for l in range(L):
            eng.mom_view(l).copy_(torch.as_tensor(g[f"m0_{l}"]))
        eng.mass[0, :L] = torch.as_tensor(g["M"], dtype=torch.float32)
    eng.moments_ready = True
    xi = pack(eng, [g[f"xi{l}"] for l in range(L)])
    xr = pack(eng, [g[f"xr{l}"] for l in range(L)]) if resample else None
    eng.step(g["X"], g["Y"], N_, lr, beta, T, resample=resample, xi=xi, xi_resample=xr)
    sfx = "r" if resample else ""
    for l in range(L):
        assert rel_err(cpu(eng.W_view(l)), g[f"W1{sfx}_{l}"]) < 1e-5
        assert rel_err(cpu(eng.mom_view(l)), g[f"m1{sfx}_{l}"]) < 1e-4


def test_config1_sgld_trajectory(dev, golden):
    """Config 1 (1-layer RBF n_rf=100, mcycle-shaped N=133, full batch): 50 SGLD steps with
    injected noise track the float64 oracle trajectory."""
    from likelihoods import Gaussian
    from models.regression_model import RegressionDGP
    g = golden("config1_sgld")
    m = RegressionDGP(1, 1, n_hidden_layers=1, n_rf=100, n_gp=1,
                      likelihood=Gaussian(variance=0.01), kernel_type_list=["RBF"])
    with torch.no_grad():
        m.BNN.layers[0].z.copy_(torch.as_tensor(g["z0"]))
        m.BNN.layers[1].assign_W(g["W0"])
        m.likelihood.lik_log_var.copy_(torch.as_tensor(g["lik_log_var"]))
    m.precond_update(None, 133, precond_type="identity")
    lr, beta, T, N_ = g["step_scalars"]
    eng = m._engine
    worst = 0.0
    for t in range(g["xi"].shape[0]):
        xi = pack(eng, [g["xi"][t]])
        m._engine.step(g["X"], g["Y"], N_, lr, beta, T, xi=xi)
        worst = max(worst, rel_err(cpu(eng.W_view(0)), g["traj"][t]))
    assert worst < 1e-4


def test_standalone_update(dev, golden):
    g = golden("rbf2_gauss")
    m = model_from_fixture(g)
    eng = m._engine
    lr, beta, T, N_ = g["step_scalars"]
    eng.mass[0, :2] = torch.as_tensor(g["M"], dtype=torch.float32)
    with torch.no_grad():
        for l in range(2):
            eng.mom_view(l).copy_(torch.as_tensor(g[f"m0_{l}"]))
    grad = pack(eng, [g["g0"], g["g1"]])
    xi = pack(eng, [g["xi0"], g["xi1"]])
    eng.sghmc_update(grad, lr, beta, T, N_, xi=xi)
    for l in range(2):
        W1, m1 = O.sghmc_update(g[f"W{l}"], g[f"m0_{l}"], g[f"g{l}"], lr, N_, beta, T,
                                g["M"][l], g[f"xi{l}"])
        assert rel_err(cpu(eng.W_view(l)), W1) < 1e-6
        assert rel_err(cpu(eng.mom_view(l)), m1) < 1e-5


def test_device_philox_noise_counter(dev, golden):
    """The update's in-kernel noise is the Philox stream (seed, sub = step, NOISE, tag = chain)
    indexed by the packed element: a Philox step equals an injected-noise step."""
    g = golden("mixed5")
    a, b = model_from_fixture(g), model_from_fixture(g)
    lr, beta, T, N_ = g["step_scalars"]
    b._engine.seed = a._engine.seed  # each model draws its own key (engine_key): share a's here
    for mm in (a, b):
        mm.precond_update(None, N_, precond_type="identity")
        mm._engine.mom.zero_()
        mm._engine.step_ctr.fill_(5)
    a._engine.step(g["X"], g["Y"], N_, lr, beta, T)
    eng = b._engine
    xi = R.philox_normal(eng.layout.w_total, eng.seed, 5, R.PURPOSE_NOISE, tag=0)
    eng.step(g["X"], g["Y"], N_, lr, beta, T,
             xi=torch.as_tensor(xi, dtype=torch.float32)[None])
    assert rel_err(cpu(a._engine.theta), cpu(eng.theta)) < 1e-5
    assert int(a._engine.step_ctr) == 6


def test_two_models_draw_independent_noise(dev):
    """Two models built in one process get distinct Philox keys (the reference's global
    tf.random.normal stream moves on between models, models/dgp.py:210-212): from identical state
    and data their SGHMC steps differ; set_seed makes the keys reproducible."""
    from dgprf import engine as E
    from likelihoods import Gaussian
    from models.regression_model import RegressionDGP
    mk = lambda: RegressionDGP(3, 1, n_hidden_layers=2, n_rf=16, n_gp=[2, 1],
                               likelihood=Gaussian(variance=0.1))
    E.set_seed(11)
    a, b = mk(), mk()
    E.set_seed(11)
    c = mk()
    assert a._engine.seed != b._engine.seed and c._engine.seed == a._engine.seed
    rng = np.random.default_rng(0)
    X = rng.standard_normal((20, 3)).astype(np.float32)
    Y = rng.standard_normal((20, 1)).astype(np.float32)
    for mm in (a, b):
        mm.precond_update(None, 100, precond_type="identity")
    for t in ("z", "theta", "mom", "hyp"):
        getattr(b._engine, t).copy_(getattr(a._engine, t))
    a.sgmcmc_update(X, Y, 100, lr=0.01)
    b.sgmcmc_update(X, Y, 100, lr=0.01)
    assert not torch.equal(a._engine.theta, b._engine.theta)


# ----------------------------------------------------------------------------- minibatching
def test_epoch_minibatch_rows_bit_exact(dev):
    """DGPRF_BATCH_EPOCH rows (device Feistel) == oracle rows: the gradient of an EPOCH batch is
    bitwise the gradient of the INDEXED batch with the oracle's indices."""
    from likelihoods import Gaussian
    from models.regression_model import RegressionDGP
    m = RegressionDGP(3, 1, n_hidden_layers=2, n_rf=24, n_gp=[4, 1], likelihood=Gaussian())
    eng = m._engine
    n, B = 1037, 50
    X = torch.randn(n, 3, device=dev)
    Y = torch.randn(n, 1, device=dev)
    iters = n // B
    for t in (0, 7, iters - 1, iters, 3 * iters + 2):
        eng.step_ctr.fill_(t)
        ge = eng.grad(X, Y, n, batch_size=B, mode=2, perm_seed=99)
        rows = R.batch_rows(t, B, n, iters, perm_seed=99)
        gi = eng.grad(X, Y, n, batch_size=B, mode=1, idx=rows.astype(np.int32))
        assert torch.equal(ge, gi), t
        gd = eng.grad(X[torch.as_tensor(rows, device=dev)], Y[torch.as_tensor(rows, device=dev)], n)
        assert torch.equal(ge, gd), t


def test_graph_replay_equals_eager_steps(dev):
    from likelihoods import Gaussian
    from models.regression_model import RegressionDGP
    from dgprf import engine as E
    E.set_seed(11)
    a = RegressionDGP(4, 1, n_hidden_layers=2, n_rf=40, n_gp=[3, 1], likelihood=Gaussian())
    E.set_seed(11)
    b = RegressionDGP(4, 1, n_hidden_layers=2, n_rf=40, n_gp=[3, 1], likelihood=Gaussian())
    assert torch.equal(a._engine.theta, b._engine.theta)
    n, B = 640, 64
    X = torch.randn(n, 4, device=dev)
    Y = torch.randn(n, 1, device=dev)
    for mm in (a, b):
        mm.precond_update(None, n, precond_type="identity")
    b._engine.mom.copy_(a._engine.mom)
    a.run_sgmcmc(X, Y, n, 24, batch_size=B, lr=0.01, momentum_decay=0.9, steps_per_graph=8,
                 perm_seed=3)
    for _ in range(24):
        b._engine.step(X, Y, n, 0.01, 0.9, 1.0, batch_size=B, mode=2, perm_seed=3)
    assert int(a._engine.step_ctr) == 24 == int(b._engine.step_ctr)
    assert torch.equal(a._engine.theta, b._engine.theta)
    assert torch.equal(a._engine.mom, b._engine.mom)


def test_per_call_sgmcmc_update_equals_graph_replays(dev):
    """The reference's driver loop — one model.sgmcmc_update(x, y, N, ...) call per minibatch
    (experiments/utils_training.py:45-61 -> models/dgp.py:184-216) — is bit-equal over 10 steps to
    run_sgmcmc's graph replays fed the same minibatch rows (the device epoch permutation, restated
    by the oracle), and builds Omega once (fixed z: only when z or a hyper-parameter is stale)."""
    from likelihoods import Gaussian
    from models.regression_model import RegressionDGP
    from dgprf import engine as E
    E.set_seed(21)
    a = RegressionDGP(8, 1, n_hidden_layers=3, n_rf=64, n_gp=[8, 8, 1], likelihood=Gaussian())
    E.set_seed(21)
    b = RegressionDGP(8, 1, n_hidden_layers=3, n_rf=64, n_gp=[8, 8, 1], likelihood=Gaussian())
    n, B, steps = 2000, 200, 10
    X = torch.randn(n, 8, device=dev)
    Y = torch.randn(n, 1, device=dev)
    for mm in (a, b):
        mm.precond_update(None, n, precond_type="identity")
    b._engine.mom.copy_(a._engine.mom)
    a.run_sgmcmc(X, Y, n, steps, batch_size=B, lr=0.01, momentum_decay=0.9, steps_per_graph=steps,
                 perm_seed=5)
    eng = b._engine
    calls = []
    orig = eng.build_omega
    eng.build_omega = lambda *args, **kw: (calls.append(1), orig(*args, **kw))[1]
    for t in range(steps):
        rows = torch.as_tensor(R.batch_rows(t, B, n, n // B, perm_seed=5), device=dev)
        b.sgmcmc_update(X[rows], Y[rows], n, lr=0.01, momentum_decay=0.9)
    assert len(calls) <= 1  # Omega built at most once over the 10 calls
    assert int(a._engine.step_ctr) == steps == int(eng.step_ctr)
    assert torch.equal(a._engine.theta, eng.theta)
    assert torch.equal(a._engine.mom, eng.mom)
    with torch.no_grad():  # a hyper-parameter write makes the next call rebuild
        b.kernel_list[1].log_inv_length_scale.sub_(0.05)
    n0 = len(calls)
    b.sgmcmc_update(X[:B], Y[:B], n, lr=0.01, momentum_decay=0.9)
    assert len(calls) == n0 + 1


def test_per_call_host_batches_equal_device_batches(dev):
    """Host minibatches (float32 / float64 numpy, CPU tensors, 1-D Y) go through the pinned
    HostStage ring (one async H2D copy per call); 14 calls — past the ring's 4 slots, with a
    larger batch mid-run that regrows it — are bit-equal to the same calls on device batches."""
    from likelihoods import Gaussian
    from models.regression_model import RegressionDGP
    from dgprf import engine as E
    E.set_seed(23)
    a = RegressionDGP(8, 1, n_hidden_layers=2, n_rf=64, n_gp=[8, 1], likelihood=Gaussian())
    E.set_seed(23)
    b = RegressionDGP(8, 1, n_hidden_layers=2, n_rf=64, n_gp=[8, 1], likelihood=Gaussian())
    n = 4000
    for mm in (a, b):
        mm.precond_update(None, n, precond_type="identity")
    b._engine.mom.copy_(a._engine.mom)
    g = torch.Generator().manual_seed(4)
    for t in range(14):
        B = 600 if t == 7 else 200
        Xh = torch.randn(B, 8, generator=g)
        Yh = torch.randn(B, generator=g)
        a.sgmcmc_update(Xh.to(dev), Yh.to(dev), n, lr=0.01, momentum_decay=0.9)
        form = t % 3
        xh = Xh.numpy() if form == 0 else (Xh.double().numpy() if form == 1 else Xh)
        yh = Yh.numpy() if form != 2 else Yh
        b.sgmcmc_update(xh, yh, n, lr=0.01, momentum_decay=0.9)
    assert b._engine._stage is not None and b._engine._stage.k == 14
    assert torch.equal(a._engine.theta, b._engine.theta)
    assert torch.equal(a._engine.mom, b._engine.mom)


def test_checkpoint_resume_bit_exact(dev, tmp_path):
    """save() at step 100 -> load() into another model (one that has already captured and replayed
    its own step graphs) -> 100 more graph-replayed steps is bitwise the 200 uninterrupted steps
    (SURVEY §5 checkpoint / resume; the reference keeps only live variable aliases,
    experiments/utils_training.py:226)."""
    from likelihoods import Gaussian
    from models.regression_model import RegressionDGP
    from dgprf import engine as E
    mk = lambda: RegressionDGP(8, 1, n_hidden_layers=3, n_rf=64, n_gp=[8, 8, 1],
                               likelihood=Gaussian())
    E.set_seed(31)
    a = mk()
    n = 3000
    X = torch.randn(n, 8, device=dev)
    Y = torch.randn(n, 1, device=dev)
    a.precond_update(None, n, precond_type="identity")
    run = dict(batch_size=200, lr=0.01, momentum_decay=0.9, steps_per_graph=50, perm_seed=4)
    a.run_sgmcmc(X, Y, n, 100, **run)
    path = str(tmp_path / "ckpt.npz")
    a.save(path)
    a.run_sgmcmc(X, Y, n, 100, **run)
    E.set_seed(999)  # a different construction draw: everything must come from the checkpoint
    b = mk()
    # b has already captured (and replayed) graphs of the same arguments under its own Philox key:
    # load() must not leave them to be replayed with the old key
    b.precond_update(None, n, precond_type="identity")
    b.run_sgmcmc(X, Y, n, 100, **run)
    assert b._engine._graphs
    b.load(path)
    assert int(b._engine.step_ctr) == 100 and b._engine.seed == a._engine.seed
    assert b.W_mcmc[0].moments is not None
    b.run_sgmcmc(X, Y, n, 100, **run)
    torch.cuda.synchronize()
    for t in ("theta", "mom", "mass", "hyp", "z", "step_ctr"):
        assert torch.equal(getattr(a._engine, t), getattr(b._engine, t)), t
    with pytest.raises(ValueError):  # a checkpoint of another shape is refused
        RegressionDGP(8, 1, n_hidden_layers=3, n_rf=32, n_gp=[8, 8, 1],
                      likelihood=Gaussian()).load(path)


def test_sgmcmc_graphs_rebuild_omega_only_when_stale(dev):
    """sgmcmc_graphs builds Omega / c / sigma^2 only when z or a hyper-parameter changed since the
    last build (torch version counters of the packed buffers): a second call with nothing changed
    builds nothing; an in-place hyper-parameter update (as the MCEM Adam applies it) or a new z
    rebuilds, and the rebuilt Omega equals a from-scratch build."""
    from likelihoods import Gaussian
    from models.regression_model import RegressionDGP
    from dgprf import engine as E
    E.set_seed(12)
    m = RegressionDGP(4, 1, n_hidden_layers=2, n_rf=40, n_gp=[3, 1], likelihood=Gaussian())
    eng = m._engine
    n = 640
    X = torch.randn(n, 4, device=dev)
    Y = torch.randn(n, 1, device=dev)
    m.precond_update(None, n, precond_type="identity")
    calls = []
    orig = eng.build_omega
    eng.build_omega = lambda *a, **k: (calls.append(1), orig(*a, **k))[1]
    run = lambda: m.run_sgmcmc(X, Y, n, 8, batch_size=64, lr=0.01, momentum_decay=0.9,
                               steps_per_graph=8)
    run()
    first = len(calls)
    run()
    assert len(calls) == first  # nothing changed: no rebuild
    with torch.no_grad():
        m.kernel_list[0].log_inv_length_scale.sub_(0.1)
        m.likelihood.lik_log_var.add_(0.05)
    run()
    assert len(calls) == first + 1
    om = torch.empty_like(eng.omega)
    orig(z=eng.z, omega=om)
    torch.cuda.synchronize()
    assert torch.equal(om, eng.omega)
    with torch.no_grad():
        m.BNN.layers[0].z.mul_(1.5)
    run()
    assert len(calls) == first + 2
    run()
    assert len(calls) == first + 2


def test_graph_fresh_z_random_fixed_false(dev):
    """random_fixed=False inside graph-replayed steps (layers/rf_layers.py:39-41): every step draws
    z ~ N(0,1) on the device from Philox (seed, sub = step, RNG_Z, tag = 1 + layer) and builds that
    step's Omega; 3 graph steps equal 3 eager steps of a random_fixed=True twin whose z is set to
    the same draws (oracle Philox) before each step."""
    from dgprf import engine as E
    from likelihoods import Gaussian
    from models.regression_model import RegressionDGP
    E.set_seed(21)
    a = RegressionDGP(3, 1, n_hidden_layers=2, n_rf=[32, 24], n_gp=[4, 1],
                      likelihood=Gaussian(variance=0.2), random_fixed=False)
    b = RegressionDGP(3, 1, n_hidden_layers=2, n_rf=[32, 24], n_gp=[4, 1],
                      likelihood=Gaussian(variance=0.2))
    n, B = 320, 32
    X = torch.randn(n, 3, device=dev)
    Y = torch.randn(n, 1, device=dev)
    for mm in (a, b):
        mm.precond_update(None, n, precond_type="identity")
    ea, eb = a._engine, b._engine
    for t in ("theta", "mom", "hyp", "step_ctr"):
        getattr(eb, t).copy_(getattr(ea, t))
    eb.seed = ea.seed
    a.run_sgmcmc(X, Y, n, 3, batch_size=B, lr=0.01, momentum_decay=0.9, steps_per_graph=3,
                 perm_seed=5)
    pl = eb.layout
    for t in range(3):
        for l in range(2):
            nz = pl.d[l] * pl.n_rf[l]
            z = R.philox_normal(nz, eb.seed, t, R.PURPOSE_Z, tag=1 + l)
            eb.z_view(l).copy_(torch.as_tensor(z.reshape(pl.d[l], pl.n_rf[l]), dtype=torch.float32))
        eb.step(X, Y, n, 0.01, 0.9, 1.0, batch_size=B, mode=2, perm_seed=5)
    assert int(ea.step_ctr) == 3 == int(eb.step_ctr)
    assert rel_err(cpu(ea.theta), cpu(eb.theta)) < 1e-5


def test_graph_fresh_z_partial_fused_forward(dev):
    """random_fixed=False on ONE layer (fresh_z = 0b010) at B = 2,048 with one chain: the step runs
    the all-layer fused forward, which reads every layer's Omega from the workspace copy — the
    fixed layers' Omega must be copied there.  3 graph steps equal 3 eager steps of a
    random_fixed=True twin whose layer-1 z is set to the device draws before each step."""
    from dgprf import _native as N
    from dgprf import engine as E
    spec = E.ModelSpec(3, 1, [N.RBF, N.ARC, N.RBF], [64, 48, 32], [4, 4, 1], False,
                       N.LIK_GAUSSIAN)
    ea = E.Engine(spec, 1, seed=777)
    ea.draw_init()
    E.normal(None, N.RNG_W, out=ea.theta)
    E.normal(None, N.RNG_MOMENTS, out=ea.mom)
    ea.build_omega()
    eb = E.Engine(spec, 1, seed=ea.seed)
    for t in ("z", "hyp", "theta", "mom", "step_ctr"):
        getattr(eb, t).copy_(getattr(ea, t))
    n, B, lr, beta, T, steps = 8192, 2048, 0.01, 0.9, 1.0, 3
    X = torch.randn(n, 3, device=dev)
    Y = torch.randn(n, 1, device=dev)
    pl, _ = ea.plan_ws(B, 0b010)
    # the all-layer fused forward of the step (step_common.h step_fused_fwd)
    assert pl.rt_per_group >= 8 and pl.n_chains == 1 and pl.a0_off < 0 and pl.omf_off >= 0
    ea.graph(X, Y, B, n, lr, beta, T, steps, perm_seed=5, fresh_z=0b010).launch()
    for t in range(steps):
        z = R.philox_normal(pl.d[1] * pl.n_rf[1], ea.seed, t, R.PURPOSE_Z, tag=1 + 1)
        eb.z_view(1).copy_(torch.as_tensor(z.reshape(pl.d[1], pl.n_rf[1]), dtype=torch.float32))
        eb.step(X, Y, n, lr, beta, T, batch_size=B, mode=N.BATCH_EPOCH, perm_seed=5)
    assert int(ea.step_ctr) == steps == int(eb.step_ctr)
    assert rel_err(cpu(ea.theta), cpu(eb.theta)) < 1e-5


def test_graph_fresh_z_two_chains(dev):
    """random_fixed=False with C = 2 chains in one graph: chain c draws its own z from Philox
    (seed, sub = step, RNG_Z, tag = 1 + l + 16 c) into its own workspace copy of Omega (chain
    stride ws_chain).  At T = 0 (no noise) each chain's 3 graph steps equal 3 eager single-chain
    steps on the same rows (oracle Feistel rows of chain c) with z set to that chain's draws."""
    from dgprf import _native as N
    from dgprf import engine as E
    from oracle import rng as R
    spec = E.ModelSpec(3, 1, [N.RBF, N.ARC], [32, 24], [4, 1], False, N.LIK_GAUSSIAN)
    two = E.Engine(spec, 2, seed=4242)
    two.draw_init()
    E.normal(None, N.RNG_W, out=two.theta)
    E.normal(None, N.RNG_MOMENTS, out=two.mom)
    two.build_omega()
    n, B, lr, beta, steps = 320, 32, 0.01, 0.9, 3
    X = torch.randn(n, 3, device=dev)
    Y = torch.randn(n, 1, device=dev)
    th0, mo0 = two.theta.clone(), two.mom.clone()
    two.graph(X, Y, B, n, lr, beta, 0.0, steps, perm_seed=7, fresh_z=0b11).launch()
    pl, ws = two.plan_ws(B, 0b11)
    iters = n // B
    for c in range(2):
        # the workspace's Omega of chain c is the last step's fresh draw
        om_ws = ws[c * pl.ws_chain + pl.omf_off:c * pl.ws_chain + pl.omf_off + pl.omega_total]
        for l in range(2):
            z = R.philox_normal(pl.d[l] * pl.n_rf[l], two.seed, steps - 1, R.PURPOSE_Z,
                                tag=1 + l + 16 * c).reshape(pl.d[l], pl.n_rf[l])
            ref = np.exp(cpu(two.lis_view(l)))[:, None] * z
            got = cpu(om_ws[pl.omega_off[l]:pl.omega_off[l] + z.size]).reshape(z.shape)
            assert rel_err(got, ref) < 1e-6, (c, l)
        one = E.Engine(spec, 1, seed=two.seed)
        one.hyp.copy_(two.hyp[:one.hyp.numel()])
        one.theta.copy_(th0[c:c + 1])
        one.mom.copy_(mo0[c:c + 1])
        for t in range(steps):
            for l in range(2):
                z = R.philox_normal(pl.d[l] * pl.n_rf[l], two.seed, t, R.PURPOSE_Z,
                                    tag=1 + l + 16 * c)
                one.z_view(l).copy_(torch.as_tensor(z.reshape(pl.d[l], pl.n_rf[l]),
                                                    dtype=torch.float32))
            rows = R.batch_rows(t, B, n, iters, perm_seed=7, chain=c).astype(np.int32)
            one.step(X, Y, n, lr, beta, 0.0, batch_size=B, mode=N.BATCH_INDEXED, idx=rows)
        assert rel_err(cpu(one.theta[0]), cpu(two.theta[c])) < 1e-5, c


def test_device_cyclical_schedule(dev):
    """DGPRF_SCHED_CYCLICAL: burn-in lr0/T=0 then lr0 * rate^2, T=1 (utils_training.py:47-61)."""
    from likelihoods import Gaussian
    from models.regression_model import RegressionDGP
    from dgprf import engine as E
    from utils import cyclical_step_rate
    E.set_seed(5)
    a = RegressionDGP(2, 1, n_hidden_layers=1, n_rf=16, n_gp=1, likelihood=Gaussian())
    E.set_seed(5)
    b = RegressionDGP(2, 1, n_hidden_layers=1, n_rf=16, n_gp=1, likelihood=Gaussian())
    n, B, start, cyc = 320, 32, 6, 5
    X = torch.randn(n, 2, device=dev)
    Y = torch.randn(n, 1, device=dev)
    for mm in (a, b):
        mm.precond_update(None, n, precond_type="identity")
    b._engine.mom.copy_(a._engine.mom)
    a.run_sgmcmc(X, Y, n, 16, batch_size=B, lr=0.05, momentum_decay=0.5, steps_per_graph=4,
                 schedule="cyclical", start_step=start, cycle_length=cyc)
    for t in range(16):
        if t < start:
            lr, T = 0.05, 0.0
        else:
            r, _ = cyclical_step_rate(t - start + 1, cyc, "cosine", min_value=0.0)
            lr, T = float(np.float32(0.05) * (r * r)), 1.0
        b._engine.step(X, Y, n, lr, 0.5, T, batch_size=B, mode=2)
    assert rel_err(cpu(a._engine.theta), cpu(b._engine.theta)) < 1e-5


def test_multichain_chain0_matches_single_chain(dev):
    from dgprf import engine as E
    from dgprf import _native as N
    spec = E.ModelSpec(3, 1, [N.RBF, N.ARC], [32, 48], [4, 1], False, N.LIK_GAUSSIAN)
    one, three = E.Engine(spec, 1, seed=42), E.Engine(spec, 3, seed=42)
    one.draw_init()
    three.z.copy_(one.z)
    three.hyp.copy_(one.hyp)
    three.theta.copy_(one.theta.expand(3, -1))
    for e in (one, three):
        e.mom.zero_()
    n, B = 512, 64
    X = torch.randn(n, 3, device=dev)
    Y = torch.randn(n, 1, device=dev)
    for e in (one, three):
        e.build_omega()
        e.graph(X, Y, B, n, 0.02, 0.9, 1.0, 6).launch()
    assert torch.equal(one.theta[0], three.theta[0])
    assert not torch.equal(three.theta[0], three.theta[1])
    assert not torch.equal(three.theta[1], three.theta[2])


# ----------------------------------------------------------------------------- predictive
def test_predictive_lse_matches_oracle(dev, golden):
    from likelihoods import Gaussian
    from models.regression_model import RegressionDGP
    from dgprf.predictive import PredictiveLSE
    g = golden("predictive")
    m = RegressionDGP(4, 1, n_hidden_layers=2, n_rf=[30, 30], n_gp=[5, 1],
                      likelihood=Gaussian(variance=float(np.exp(g["lik_log_var"]))),
                      set_nonzero_mean=True)
    g2 = dict(g)
    g2["kinds"] = np.array([0, 0])
    load_params(m, g2)
    acc = PredictiveLSE(m._engine, g["Xt"], g["Yt"])
    S = g["logp"].shape[0]
    for s in range(S):
        m.assign_W([g[f"Ws{s}_0"], g[f"Ws{s}_1"]])
        lp, se = m.eval_log_likelihood_and_se([(g["Xt"], g["Yt"])])
        assert np.max(np.abs(cpu(lp) - g["logp"][s])) < 1e-4
        acc.add_sample()
    ll, rmse = acc.finalize(y_std=float(g["y_std"]))
    assert abs(ll - float(g["LL"])) < 1e-4      # north_star: predictive log-lik within 1e-4
    assert abs(rmse - float(g["RMSE"])) < 1e-5 * max(1.0, float(g["RMSE"]))


def test_precond_rmsprop_masses(dev, golden):
    from likelihoods import Gaussian
    from models.regression_model import RegressionDGP
    g = golden("precond")
    for centered, key in ((False, "M"), (True, "M_centered")):
        m = RegressionDGP(2, 1, n_hidden_layers=2, n_rf=[16, 24], n_gp=[3, 1],
                          likelihood=Gaussian(variance=float(np.exp(g["lik_log_var"]))),
                          set_nonzero_mean=True)
        g2 = dict(g)
        g2["kinds"] = np.array([0, 0])
        load_params(m, g2)
        m.precond_update(None, int(g["N"]), precond_type="identity")
        m0 = cpu(m._engine.mom).copy()
        ds = [(g["Xs"][k], g["Ys"][k]) for k in range(4)]
        m.precond_update(ds, int(g["N"]), K_batches=4, second_moment_centered=centered)
        M = cpu(m._engine.mass)[0]
        assert rel_err(M, g[key]) < 1e-4
        for l in range(2):   # moments = sqrt(M) * rsqrt(1) * moments_before
            o, n_ = m._engine.layout.w_off[l], m._engine.layout.P[l] * m._engine.layout.n_gp[l]
            assert rel_err(cpu(m._engine.mom)[0, o:o + n_], np.sqrt(M[l]) * m0[0, o:o + n_]) < 1e-5
        with pytest.raises(AssertionError):
            m.precond_update(ds[:2], int(g["N"]), K_batches=4)


# ----------------------------------------------------------------------------- edge shapes
@pytest.mark.parametrize("kinds,n_rf,n_gp,d_in,cat,lik,B", [
    (["RBF"], [1], [1], 1, False, "gaussian", 1),            # smallest everything
    (["RBF", "RBF"], [100, 17], [30, 2], 100, False, "gaussian", 33),  # large-d path, 2 out tiles
    (["ARC", "RBF"], [64, 64], [16, 5], 40, True, "softmax", 200),      # input_cat, wide d
    (["RBF"] * 3, [1024] * 3, [8, 8, 1], 8, False, "gaussian", 200),   # config 2 shapes
    # n_rf 4096: 8-wave whole-slice backward, gW tiles of g % 16 != 0 staged through LDS (g = 10,
    # 2, 48), a d > 32 hidden layer (KS = 0), and g = 60, whose staging does not fit next to the
    # slice image (the 4-wave form instead)
    (["ARC", "RBF"], [4096, 4096], [10, 2], 6, False, "gaussian", 64),
    (["RBF", "RBF"], [4096, 4096], [48, 3], 12, False, "gaussian", 40),
    (["RBF"], [4096], [60], 5, False, "softmax", 20),
])
def test_edge_shapes_forward_and_grad(dev, kinds, n_rf, n_gp, d_in, cat, lik, B):
    from likelihoods import Gaussian, Softmax
    from models.dgp import DGP_RF
    rng = np.random.default_rng(B + d_in)
    d_out = n_gp[-1]
    m = DGP_RF(d_in, d_out, n_hidden_layers=len(kinds), n_rf=n_rf, n_gp=n_gp,
               likelihood=Gaussian() if lik == "gaussian" else Softmax(),
               kernel_type_list=kinds, input_cat=cat)
    p = O.Params(d_in, d_out, n_rf, n_gp, kinds, lik, cat,
                 z=[cpu(m.BNN.layers[2 * l].z) for l in range(len(kinds))],
                 W=[cpu(w) for w in m.W_mcmc],
                 log_inv_ls=[cpu(k.log_inv_length_scale) for k in m.kernel_list],
                 lik_log_var=np.log(0.1))
    X = rng.standard_normal((B, d_in))
    Y = rng.standard_normal((B, d_out)) if lik == "gaussian" else \
        rng.integers(0, d_out, (B, 1)).astype(float)
    assert rel_err(cpu(m.BNN(X)), O.forward(p, X)) < 5e-5
    G = unpack(m._engine, m._engine.grad(X, Y, 10_000))
    ref = O.grad_W(p, X, Y, 10_000)
    for l in range(len(kinds)):
        assert rel_err(G[l], ref[l]) < 2e-4, l


def test_api_errors(dev):
    from likelihoods import Gaussian
    from models.regression_model import RegressionDGP
    m = RegressionDGP(3, 1, n_hidden_layers=1, n_rf=8, n_gp=1, likelihood=Gaussian())
    X, Y = np.zeros((4, 3), np.float32), np.zeros((4, 1), np.float32)
    with pytest.raises(AssertionError, match="moments"):
        m.sgmcmc_update(X, Y, 100)
    m.precond_update(None, 100, precond_type="identity")
    with pytest.raises(AssertionError, match="moments"):   # hyper-parameters have no moments yet
        m.sgmcmc_update(X, Y, 100, full_bayesian=True)
    with pytest.raises(ValueError):
        m.sgmcmc_update(np.zeros((4, 2), np.float32), Y, 100)
    with pytest.raises(NotImplementedError):
        m.precond_update(None, 100, precond_type="adam")
    m.sgmcmc_update(X, Y, 100)   # works after precond_update
    assert torch.isfinite(m._engine.theta).all()


# ----------------------------------------------------------------------------- statistics
@pytest.mark.parametrize("beta", [0.0, 0.9])
def test_sampler_targets_gaussian_posterior(dev, beta):
    """Full-batch SGLD / SGHMC on a 1-layer RF model (fixed features, Gaussian likelihood):
    the posterior of W is N(mu, Sigma), Lambda = I + Phi^T Phi / s2, mu = Lambda^-1 Phi^T y / s2.
    Sample moments from the device Philox-driven chain match it."""
    from likelihoods import Gaussian
    from models.regression_model import RegressionDGP
    from dgprf import engine as E
    E.set_seed(1000 + int(beta * 10))
    n, R_, s2 = 64, 4, 0.5
    m = RegressionDGP(1, 1, n_hidden_layers=1, n_rf=R_, n_gp=1, likelihood=Gaussian(variance=s2))
    rng = np.random.default_rng(0)
    X = rng.uniform(-2, 2, (n, 1))
    Y = np.sin(2 * X) + 0.3 * rng.standard_normal((n, 1))
    Phi = cpu(m.BNN.layers[0](X)).astype(np.float64)
    Lam = np.eye(2 * R_) + Phi.T @ Phi / s2
    Sig = np.linalg.inv(Lam)
    mu = Sig @ Phi.T @ Y[:, 0] / s2
    m.precond_update(None, n, precond_type="identity")
    eps = 0.02 * np.min(np.diag(Sig))          # Langevin step h^2 = lr / N
    lr = eps * n
    Xd = torch.as_tensor(X, dtype=torch.float32, device=dev)
    Yd = torch.as_tensor(Y, dtype=torch.float32, device=dev)
    thin = 25
    m.run_sgmcmc(Xd, Yd, n, 2000, batch_size=n, lr=lr, momentum_decay=beta, steps_per_graph=thin)
    samples = []
    for _ in range(2000):
        m.run_sgmcmc(Xd, Yd, n, thin, batch_size=n, lr=lr, momentum_decay=beta,
                     steps_per_graph=thin)
        samples.append(m._engine.W_view(0)[:, 0].clone())
    S = torch.stack(samples).double().cpu().numpy()
    sd = np.sqrt(np.diag(Sig))
    z = (S.mean(0) - mu) / sd
    assert np.max(np.abs(z)) < 0.35, z                 # mean within 0.35 posterior sd
    ratio = S.std(0) / sd
    assert np.all((ratio > 0.8) & (ratio < 1.2)), ratio


def test_sgld_demo_two_mode_mixture(dev):
    """SURVEY §4's reference-held statistical target, experiments/SGLD-demo.ipynb cells 2-3: SGLD on
    the 1-D mixture 0.5 N(-2, 2) + 0.5 N(2, 0.2), x0 = 5, lr_t = 0.1 (1 + t)^-0.55,
    x <- x + lr grad log p + sqrt(2 lr) eps — "to see whether SGLD can find two modes".  The update
    is the device SGHMC kernel (dgprf_sghmc_update, beta = 0, T = 1, M = 1, data_size = 1: the
    reference's m = -hNg + sqrt(2) xi, theta += h m with h = sqrt(lr), models/dgp.py:206-216) on
    8,192 independent particles (2,048 chains x 4 packed parameters) driven by its Philox noise,
    the gradient of -log p supplied per step.  After 20,000 steps both modes hold particles, and the
    ensemble matches a float64 numpy run of the same dynamics (independent noise) to the sampling
    error of the particle count: fraction left of the barrier within 0.03, mean within 0.12, variance
    within 10 %."""
    from dgprf import engine as E
    from dgprf import _native as N
    m1, v1, m2, v2 = -2.0, 2.0, 2.0, 0.2

    def grad_log_p(x, xp):
        a = 0.5 * xp.exp(-0.5 * (x - m1) ** 2 / v1) / np.sqrt(2 * np.pi * v1)
        b = 0.5 * xp.exp(-0.5 * (x - m2) ** 2 / v2) / np.sqrt(2 * np.pi * v2)
        return (a * (-(x - m1) / v1) + b * (-(x - m2) / v2)) / (a + b)

    E.set_seed(77)
    eng = E.Engine(E.ModelSpec(1, 1, [N.RBF], [2], [1]), 2048)
    assert eng.layout.w_total == 4 and eng.per_chain_hyp is False
    eng.theta.fill_(5.0)
    eng.mom.zero_()
    steps = 20_000
    for t in range(steps):
        lr = 0.1 * (1 + t) ** -0.55
        g = -grad_log_p(eng.theta, torch)  # dU/dx with U = -log p
        eng.sghmc_update(g, lr, 0.0, 1.0, 1.0)
        eng.step_ctr += 1  # a fresh Philox counter (noise) per step
    x = eng.theta.double().cpu().numpy().reshape(-1)
    rng = np.random.default_rng(5)
    y = np.full(x.size, 5.0)
    for t in range(steps):
        lr = 0.1 * (1 + t) ** -0.55
        y = y + lr * grad_log_p(y, np) + np.sqrt(2 * lr) * rng.standard_normal(y.size)
    assert np.isfinite(x).all()
    left, left_ref = np.mean(x < 0.5), np.mean(y < 0.5)
    assert 0.25 < left < 0.6, left  # both modes found
    assert abs(left - left_ref) < 0.03, (left, left_ref)
    assert abs(x.mean() - y.mean()) < 0.12, (x.mean(), y.mean())
    assert abs(x.var() / y.var() - 1) < 0.1, (x.var(), y.var())


def test_full_config2_properties(dev):
    """Config 2 at full size (N = 1e6, B = 200, L = 3, n_rf = 1024): one step's gradient vs the
    float64 oracle on the same batch, deterministic replays, finite chains."""
    from likelihoods import Gaussian
    from models.regression_model import RegressionDGP
    from dgprf import engine as E
    from dgprf.data import regression_data
    X, Y, _ = regression_data(1_000_000, 8, seed=0, device=dev)
    runs = []
    for rep in range(2):
        E.set_seed(2)
        m = RegressionDGP(8, 1, n_hidden_layers=3, n_rf=1024, n_gp=[8, 8, 1],
                          likelihood=Gaussian(variance=0.1))
        m.precond_update(None, 1_000_000, precond_type="identity")
        if rep == 0:
            eng = m._engine
            eng.step_ctr.fill_(123)
            G = unpack(eng, eng.grad(X, Y, 1_000_000, batch_size=200, mode=2, perm_seed=0))
            rows = R.batch_rows(123, 200, 1_000_000, 5000, perm_seed=0)
            p = O.Params(8, 1, [1024] * 3, [8, 8, 1], ["RBF"] * 3,
                         z=[cpu(m.BNN.layers[2 * l].z) for l in range(3)],
                         W=[cpu(w) for w in m.W_mcmc],
                         log_inv_ls=[cpu(k.log_inv_length_scale) for k in m.kernel_list],
                         lik_log_var=np.log(0.1))
            ref = O.grad_W(p, cpu(X[torch.as_tensor(rows, device=dev)]),
                           cpu(Y[torch.as_tensor(rows, device=dev)]), 1_000_000)
            for l in range(3):
                assert rel_err(G[l], ref[l]) < 1e-4
            eng.step_ctr.fill_(0)
        m.run_sgmcmc(X, Y, 1_000_000, 500, batch_size=200, lr=0.01, momentum_decay=0.9)
        runs.append(m._engine.theta.clone())
        assert torch.isfinite(runs[-1]).all()
    assert torch.equal(runs[0], runs[1])


def test_softmax_label_outside_classes_is_nan(dev):
    """int32(Y[:, 0]) outside [0, C) (likelihoods/softmax.py:14; TF raises on it) poisons log p
    and the gradient with NaN instead of being scored as a clamped class."""
    from likelihoods import Softmax
    from models.dgp import DGP_RF
    m = DGP_RF(3, 4, n_hidden_layers=1, n_rf=16, n_gp=4, likelihood=Softmax())
    X = np.random.default_rng(0).standard_normal((5, 3)).astype(np.float32)
    Y = np.array([[0], [3], [4], [-1], [2.7]], np.float32)
    lp = cpu(m.log_likelihood(X, Y))
    assert np.isfinite(lp[[0, 1, 4]]).all() and np.isnan(lp[[2, 3]]).all()
    assert np.isnan(cpu(m._engine.grad(X, Y, 100))).any()
    assert np.isfinite(cpu(m._engine.grad(X[[0, 1, 4]], Y[[0, 1, 4]], 100))).all()
