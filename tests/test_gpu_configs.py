"""BASELINE.json configs 3-5 as parity cases: the full model shapes (layer kinds, n_rf, widths,
likelihood) with batches / test sets small enough for the float64 oracle.

  config 3: 3-layer ARC, n_rf=2048, g=[9,9,1], D=9 (protein-shaped), Gaussian
  config 4: 4-layer RBF, n_rf=4096, g=[30,30,30,10], D=784 (MNIST-shaped), softmax
  config 5: 5-layer [RBF,ARC,RBF,ARC,RBF], n_rf=8192, g=[16,16,16,16,1], D=16, Gaussian

Tolerances (fp32 device vs float64 oracle): forward / log p 5e-5 of the output scale (1e-4 for the
K = 8192-long contractions of config 4), W gradients 2e-4 of the gradient scale, one injected-noise
SGHMC update 2e-5; per-row predictive log p 2e-5 of the log p scale (an untrained random model's
log p reaches |log p| ~ 80 here, so an absolute 1e-4 would ask for 1e-6 relative).

ARC layers' relu has a kink: an inner product A within fp32 rounding (~1e-6) of 0 may take either
side in fp32 (device or numpy alike), flipping 1[A > 0] and one term of every gradient below that
layer by c dPhi.  Gradient / update cases therefore use rows whose float64 A stays >= 1e-5 from 0
in every ARC layer (`_rows_off_kinks`); the forward itself is continuous there and is not filtered.
"""
import numpy as np
import pytest
import torch

from oracle import dgp_oracle as O
from test_gpu_parity import cpu, dev, pack, rel_err, unpack  # noqa: F401

pytestmark = pytest.mark.gpu

CONFIGS = {
    2: dict(kinds=["RBF"] * 3, n_rf=[1024] * 3, n_gp=[8, 8, 1], D=8, lik="gaussian", B=64,
            n_test=500, ftol=5e-5),
    3: dict(kinds=["ARC"] * 3, n_rf=[2048] * 3, n_gp=[9, 9, 1], D=9, lik="gaussian", B=64,
            n_test=500, ftol=5e-5),
    4: dict(kinds=["RBF"] * 4, n_rf=[4096] * 4, n_gp=[30, 30, 30, 10], D=784, lik="softmax", B=32,
            n_test=64, ftol=1e-4),
    5: dict(kinds=["RBF", "ARC", "RBF", "ARC", "RBF"], n_rf=[8192] * 5, n_gp=[16, 16, 16, 16, 1],
            D=16, lik="gaussian", B=48, n_test=300, ftol=5e-5),
}


def _model(c, seed):
    from dgprf import engine as E
    from likelihoods import Gaussian, Softmax
    from models.dgp import DGP_RF
    E.set_seed(seed)
    d_out = c["n_gp"][-1]
    m = DGP_RF(c["D"], d_out, n_hidden_layers=len(c["kinds"]), n_rf=c["n_rf"], n_gp=c["n_gp"],
               likelihood=Gaussian(variance=0.1) if c["lik"] == "gaussian" else Softmax(),
               kernel_type_list=c["kinds"])
    p = O.Params(c["D"], d_out, c["n_rf"], c["n_gp"], c["kinds"], c["lik"], False,
                 z=[cpu(m.BNN.layers[2 * l].z) for l in range(len(c["kinds"]))],
                 W=[cpu(w) for w in m.W_mcmc],
                 log_inv_ls=[cpu(k.log_inv_length_scale) for k in m.kernel_list],
                 lik_log_var=np.log(0.1))
    return m, p


def _data(c, n, seed):
    rng = np.random.default_rng(seed)
    d_out = c["n_gp"][-1]
    if c["lik"] == "softmax":
        X = rng.uniform(-0.5, 0.5, (n, c["D"]))  # normalize_MNIST range
        Y = rng.integers(0, d_out, (n, 1)).astype(float)
    else:
        X = rng.standard_normal((n, c["D"]))
        Y = rng.standard_normal((n, d_out))
    return X.astype(np.float32).astype(np.float64), Y.astype(np.float32).astype(np.float64)


def _rows_off_kinks(c, p, X, Y, n, tau=1e-5):
    """The first n rows whose ARC-layer inner products all satisfy |A| >= tau (float64 oracle)."""
    _, cache = O.forward(p, X, keep=True)
    ok = np.ones(X.shape[0], dtype=bool)
    for l, k in enumerate(c["kinds"]):
        if k == "ARC":
            ok &= np.min(np.abs(cache[l][1]), axis=1) >= tau
    idx = np.nonzero(ok)[0][:n]
    assert len(idx) == n, "not enough rows away from the relu kink"
    return X[idx], Y[idx]


@pytest.mark.parametrize("cfg", [3, 4, 5])
def test_config_forward_and_grad(dev, cfg):
    c = CONFIGS[cfg]
    m, p = _model(c, 10 + cfg)
    X, Y = _data(c, 2 * c["B"], cfg)
    X, Y = _rows_off_kinks(c, p, X, Y, c["B"])
    F = cpu(m.BNN(X))
    assert rel_err(F, O.forward(p, X)) < c["ftol"]
    lp = cpu(m.log_likelihood(X, Y))
    ref_lp = O.log_prob(p, O.forward(p, X), Y)
    assert np.max(np.abs(lp - ref_lp)) < c["ftol"] * max(1.0, np.max(np.abs(ref_lp)))
    N_ = 45_730 if cfg == 3 else (60_000 if cfg == 4 else 10_000_000)
    G = unpack(m._engine, m._engine.grad(X, Y, N_))
    ref = O.grad_W(p, X, Y, N_)
    for l in range(len(c["kinds"])):
        assert rel_err(G[l], ref[l]) < 2e-4, (cfg, l)


@pytest.mark.parametrize("C", [4, 16])
@pytest.mark.parametrize("cfg", [2, 3, 4, 5])
def test_multichain_wide_slices_grad(dev, cfg, C):
    """From 4 / 16 chains per launch the plan takes wider feature slices than one chain (>= 4 / 8
    16-feature chunks per wave, dgprf_plan_init): chain 0 (the one-chain model's W) gives the
    one-chain gradient to float tolerance (another summation order), and the last chain (its W
    scaled) matches the float64 oracle."""
    import copy
    from dgprf import engine as E
    c = CONFIGS[cfg]
    L = len(c["kinds"])
    m, p = _model(c, 30 + cfg)
    X, Y = _data(c, 2 * c["B"], cfg)
    X, Y = _rows_off_kinks(c, p, X, Y, c["B"])
    N_ = {2: 1_000_000, 3: 45_730, 4: 60_000, 5: 10_000_000}[cfg]
    one = m._engine
    mc = E.Engine(one.spec, C, seed=one.seed)
    chunks = [(r + 15) // 16 for r in c["n_rf"]]
    want = [max((k + 63) // 64, min(8 if C >= 16 and g <= 16 else 4, (k + 3) // 4))
            for k, g in zip(chunks, c["n_gp"])]
    assert list(mc.layout.cpw[:L]) == want
    # 16 chains of wide layers (configs 4 / 5): one row group per chain in the backward
    pl = mc.plan_ws(c["B"])[0]
    assert (pl.rt_per_group == pl.n_row_tiles > 1) == (C >= 16 and cfg in (4, 5))
    mc.z.copy_(one.z)
    mc.hyp.copy_(one.hyp)
    mc.lik_log_var_source = one.lik_log_var_source
    s_last = 1.0 + 0.05 * (C - 1)
    scale = 1.0 + 0.05 * torch.arange(C, device=dev, dtype=torch.float32)[:, None]
    mc.theta.copy_(one.theta[:1] * scale)
    mc.init_moments()
    mc.build_omega()
    Xd = torch.as_tensor(X, dtype=torch.float32, device=dev)
    Yd = torch.as_tensor(Y, dtype=torch.float32, device=dev)
    G1 = one.grad(Xd, Yd, N_)
    G = mc.grad(Xd, Yd, N_)
    assert torch.isfinite(G).all()
    assert rel_err(cpu(G[0]), cpu(G1[0])) < 2e-5
    pc = copy.copy(p)
    pc.W = [w * np.float64(np.float32(s_last)) for w in p.W]
    ref = O.grad_W(pc, X, Y, N_)
    Gl = unpack(mc, G, chain=C - 1)
    for l in range(L):
        assert rel_err(Gl[l], ref[l]) < 2e-4, (cfg, C, l)


@pytest.mark.parametrize("cfg", [2, 3])
@pytest.mark.parametrize("path", ["tile", "rows16", "rows8", "rows"])
def test_predictive_paths_small_test_set(dev, path, cfg):
    """Config 3's model (ARC, d 9: 4 k-steps) and config 2's (RBF, d 8: 2 k-steps) on 1,001 test
    rows (a ragged tile) through the tile kernel (one wave per 16-row tile), the 16-wave row kernel
    (the product choice below 16k rows while the tiles fit the CUs), the 8-wave (past that) and the 4-wave row kernels: per-row log p
    against the oracle."""
    from dgprf import _native as N
    c = CONFIGS[cfg]
    m, p = _model(c, 33)
    Xt, Yt = _data(c, 1001, 203)
    m._engine.set_forward_path({"tile": N.FWD_TILE, "rows16": N.FWD_ROWS16, "rows8": N.FWD_ROWS8,
                                "rows": N.FWD_ROWS}[path])
    lp = cpu(m._engine.forward(Xt, Yt, logp=True)["logp"][0])
    ref = O.log_prob(p, O.forward(p, Xt), Yt)
    assert np.max(np.abs(lp - ref)) < 2e-5 * max(1.0, np.max(np.abs(ref)))


@pytest.mark.parametrize("cfg,n", [(3, 4573), (2, 5001)])
def test_predictive_two_tile_rows(dev, cfg, n):
    """The default path of one sample once the 16-row tiles outnumber the CUs (config 3's 4,573
    test rows: 286 tiles): the row kernel with two tiles per 16-wave workgroup (forward_cfg rows_tt
    = 2), whose last workgroup holds a ragged tile (and for 5,001 rows an empty one); per-row log p
    against the oracle, and equal to the one-tile 8-wave and 16-wave workgroups to fp32 rounding."""
    from dgprf import _native as N
    c = CONFIGS[cfg]
    m, p = _model(c, 35)
    Xt, Yt = _data(c, n, 205)
    lp = cpu(m._engine.forward(Xt, Yt, logp=True)["logp"][0])
    ref = O.log_prob(p, O.forward(p, Xt), Yt)
    assert np.max(np.abs(lp - ref)) < 2e-5 * max(1.0, np.max(np.abs(ref)))
    m._engine.set_forward_path(N.FWD_ROWS8)
    lp8 = cpu(m._engine.forward(Xt, Yt, logp=True)["logp"][0])
    assert np.max(np.abs(lp - lp8)) < 2e-5 * max(1.0, np.max(np.abs(ref)))
    m._engine.set_forward_path(N.FWD_ROWS16)
    lp16 = cpu(m._engine.forward(Xt, Yt, logp=True)["logp"][0])
    assert np.max(np.abs(lp - lp16)) < 2e-5 * max(1.0, np.max(np.abs(ref)))


def test_predictive_multi_round_rows(dev):
    """Config 2's shape (3-layer RBF, n_rf 1024, g [8,8,1]) over 70,001 test rows: more tiles than
    one round of resident waves (65,536 rows on 256 CUs) plus a ragged remainder; per-row log p
    against the oracle, and bit-identical on a second launch."""
    c = dict(kinds=["RBF"] * 3, n_rf=[1024] * 3, n_gp=[8, 8, 1], D=8, lik="gaussian")
    m, p = _model(c, 61)
    Xt, Yt = _data(c, 70_001, 62)
    lp = cpu(m._engine.forward(Xt, Yt, logp=True)["logp"][0])
    ref = O.log_prob(p, O.forward(p, Xt), Yt)
    assert np.max(np.abs(lp - ref)) < 2e-5 * max(1.0, np.max(np.abs(ref)))
    assert np.array_equal(lp, cpu(m._engine.forward(Xt, Yt, logp=True)["logp"][0]))


@pytest.mark.parametrize("cfg", [3, 4, 5])
def test_config_sghmc_step_injected_noise(dev, cfg):
    """One SGHMC step with injected noise at the config's full model shape; config 4 at its
    benchmarked B = 200 (the A_1 GEMM step path, align32(B) = 224: ragged 32-row GEMM tiles)."""
    c = CONFIGS[cfg]
    B = 200 if cfg == 4 else c["B"]
    m, p = _model(c, 20 + cfg)
    eng = m._engine
    X, Y = _data(c, 2 * B, 100 + cfg)
    X, Y = _rows_off_kinks(c, p, X, Y, B)
    L = len(c["kinds"])
    rng = np.random.default_rng(cfg)
    m.precond_update(None, 1000, precond_type="identity")
    m0 = [cpu(eng.mom_view(l)).astype(np.float64) for l in range(L)]
    xi = [rng.standard_normal(w.shape) for w in p.W]
    eng.step(X, Y, 1000, 0.01, 0.9, 1.0, xi=pack(eng, xi))
    O.sgmcmc_step(p, m0, X, Y, 1000, 0.01, 0.9, 1.0, [1.0] * L, xi)
    for l in range(L):
        assert rel_err(cpu(eng.W_view(l)), p.W[l]) < 2e-5, (cfg, l)


@pytest.mark.parametrize("cfg", [3, 4, 5])
def test_config_predictive_rows(dev, cfg):
    """eval_log_likelihood(_and_se) over a test set against the oracle, row by row (tile kernel for
    every config; config 4's 784-wide first layer through the A_1 GEMM, read by the tile kernel's
    WIDE layer 0)."""
    c = CONFIGS[cfg]
    m, p = _model(c, 30 + cfg)
    Xt, Yt = _data(c, c["n_test"], 200 + cfg)
    out = m._engine.forward(Xt, Yt, logp=True)
    lp = cpu(out["logp"][0])
    ref = O.log_prob(p, O.forward(p, Xt), Yt)
    assert np.max(np.abs(lp - ref)) < 2e-5 * max(1.0, np.max(np.abs(ref)))


@pytest.mark.parametrize("cfg,n_test", [(3, 4573), (4, 1000), (5, 700)])
def test_config_predictive_samples_one_launch_bit_equal(dev, cfg, n_test):
    """dgprf_forward_samples with the scratch of dgprf_forward_samples_scratch scores S samples in
    ONE launch of the one-sample predictive kernel (grid.z = sample; config 4 reading the resident
    X Omega_1), per-row log p / se to scratch, then k_lse_fold_samples in sample order; without
    that scratch it launches once per sample and folds in the kernel.  Same bits; and the summed
    result agrees with the oracle's log-sum-exp of the S samples per row."""
    from dgprf import _native as N
    from dgprf import engine as E
    from dgprf.engine import ops
    c = CONFIGS[cfg]
    m, p = _model(c, 50 + cfg)
    eng = m._engine
    Xt, Yt = _data(c, n_test, 300 + cfg)
    Xd = torch.tensor(Xt, dtype=torch.float32, device=dev)
    Yd = torch.tensor(Yt, dtype=torch.float32, device=dev)
    E.set_seed(51)
    S = 3
    thetas = torch.stack([E.normal((1, eng.layout.w_total), N.RNG_W) for _ in range(S)])
    eng.build_omega()
    a1 = eng.dataset_a1(Xd)
    assert (a1 is not None) == (cfg == 4)
    scr = eng.forward_scratch(n_test, S)
    assert scr is not None and scr.numel() >= S * n_test
    outs = []
    assert a1 is not None or eng.forward_scratch(n_test) is None  # no A_1 chunks needed
    for sc in (scr, None):
        acc = [torch.full((1, n_test), -np.inf, device=dev), torch.zeros(1, n_test, device=dev),
               torch.zeros(1, n_test, device=dev) if c["lik"] == "gaussian" else None]
        ops().forward_samples(eng._plan_t(eng.layout), thetas, eng.omega, eng.der, Xd, a1, Yd,
                              acc[0], acc[1], acc[2], sc)
        torch.cuda.synchronize()
        outs.append([cpu(a) for a in acc if a is not None])
    for a, b in zip(outs[0], outs[1]):
        assert np.array_equal(a, b), cfg
    lps = []
    for j in range(S):
        W = unpack(eng, thetas[j])
        pj = O.Params(p.d_in, p.d_out, p.n_rf, p.n_gp, p.kinds, p.likelihood, False, z=p.z, W=W,
                      log_inv_ls=p.log_inv_ls, lik_log_var=p.lik_log_var)
        lps.append(O.log_prob(pj, O.forward(pj, Xt), Yt))
    lps = np.stack(lps)
    mx = lps.max(axis=0)
    ref = mx + np.log(np.exp(lps - mx).sum(axis=0))
    got = outs[0][0][0] + np.log(outs[0][1][0])
    assert np.max(np.abs(got - ref)) < 2e-5 * max(1.0, np.max(np.abs(ref))), cfg


@pytest.mark.parametrize("cfg,n_test", [(3, 1001), (4, 960)])
def test_predictive_many_samples_take_tiles(dev, cfg, n_test):
    """One launch scoring S samples of n rows with n S >= 65,536 (forward_cfg counts every row of
    the launch) takes the tile kernel although one sample's rows are below its threshold (config
    3) or its layers have g > 16 (config 4, whose one-sample launches keep the row kernel): the
    log-sum-exp accumulators agree with the 4-wave row kernel's (FWD_ROWS pinned) to fp32
    rounding, and for config 3 with the oracle's log-sum-exp of the S samples per row."""
    from dgprf import _native as N
    from dgprf import engine as E
    from dgprf.engine import ops
    c = CONFIGS[cfg]
    m, p = _model(c, 70 + cfg)
    eng = m._engine
    Xt, Yt = _data(c, n_test, 400 + cfg)
    Xd = torch.tensor(Xt, dtype=torch.float32, device=dev)
    Yd = torch.tensor(Yt, dtype=torch.float32, device=dev)
    E.set_seed(71)
    S = 70
    assert n_test * S >= 65536
    thetas = torch.stack([E.normal((1, eng.layout.w_total), N.RNG_W) for _ in range(S)])
    eng.build_omega()
    a1 = eng.dataset_a1(Xd)
    gauss = c["lik"] == "gaussian"

    def lse():
        scr = eng.forward_scratch(n_test, S)
        acc = [torch.full((1, n_test), -np.inf, device=dev), torch.zeros(1, n_test, device=dev),
               torch.zeros(1, n_test, device=dev) if gauss else None]
        ops().forward_samples(eng._plan_t(eng.layout), thetas, eng.omega, eng.der, Xd, a1, Yd,
                              acc[0], acc[1], acc[2], scr)
        torch.cuda.synchronize()
        return cpu(acc[0])[0] + np.log(cpu(acc[1])[0])

    got = lse()
    eng.set_forward_path(N.FWD_ROWS)
    rows = lse()
    eng.set_forward_path(N.FWD_AUTO)
    assert np.all(np.isfinite(got))
    assert np.max(np.abs(got - rows)) < 2e-5 * max(1.0, np.max(np.abs(rows))), cfg
    if cfg == 3:
        lps = []
        for j in range(S):
            W = unpack(eng, thetas[j])
            pj = O.Params(p.d_in, p.d_out, p.n_rf, p.n_gp, p.kinds, p.likelihood, False, z=p.z,
                          W=W, log_inv_ls=p.log_inv_ls, lik_log_var=p.lik_log_var)
            lps.append(O.log_prob(pj, O.forward(pj, Xt), Yt))
        lps = np.stack(lps)
        mx = lps.max(axis=0)
        ref = mx + np.log(np.exp(lps - mx).sum(axis=0))
        assert np.max(np.abs(got - ref)) < 2e-5 * max(1.0, np.max(np.abs(ref)))


@pytest.mark.parametrize("cfg", [3, 4, 5])
def test_config_graph_steps_finite_and_deterministic(dev, cfg):
    """200 graph-replayed steps with on-device minibatches of B = 200 at the config's N (config 5
    scaled to N = 2e5 rows to bound memory in the test): finite, and bit-identical on replay."""
    c = CONFIGS[cfg]
    n = {3: 45_730, 4: 60_000, 5: 200_000}[cfg]
    if c["lik"] == "softmax":
        X = torch.rand(n, c["D"], device=dev) - 0.5
        Y = torch.randint(0, c["n_gp"][-1], (n, 1), device=dev).float()
    else:
        X = torch.randn(n, c["D"], device=dev)
        Y = torch.randn(n, 1, device=dev)
    out = []
    for _ in range(2):
        m, _ = _model(c, 40 + cfg)
        m.precond_update(None, n, precond_type="identity")
        m.run_sgmcmc(X, Y, n, 200, batch_size=200, lr=0.01, momentum_decay=0.9)
        out.append(m._engine.theta.clone())
        assert torch.isfinite(out[-1]).all()
    assert torch.equal(out[0], out[1])


@pytest.mark.parametrize("chunk_rows", [0, 64])
def test_wide_first_layer_forward_chunks(dev, chunk_rows):
    """Wide first layer (d = 40 > 32): the A_1 GEMM + tile kernel, in one chunk and in 64-row chunks
    (plan.agemm_chunk_rows) over a ragged 201-row set, through the row kernel (FWD_ROWS) and with
    layer 0 contracted in-kernel (FWD_NO_AGEMM); per-layer F and the LSE accumulators against the
    oracle."""
    from dgprf import _native as N
    from dgprf import engine as E
    from dgprf.predictive import PredictiveLSE
    from likelihoods import Gaussian
    from models.dgp import DGP_RF
    E.set_seed(51)
    kinds, n_rf, n_gp = ["RBF", "ARC", "RBF"], [96, 64, 48], [12, 6, 2]
    m = DGP_RF(40, 2, n_hidden_layers=3, n_rf=n_rf, n_gp=n_gp, likelihood=Gaussian(variance=0.2),
               kernel_type_list=kinds)
    p = O.Params(40, 2, n_rf, n_gp, kinds, "gaussian", False,
                 z=[cpu(m.BNN.layers[2 * l].z) for l in range(3)], W=[cpu(w) for w in m.W_mcmc],
                 log_inv_ls=[cpu(k.log_inv_length_scale) for k in m.kernel_list],
                 lik_log_var=np.log(0.2))
    rng = np.random.default_rng(8)
    X = rng.standard_normal((201, 40)).astype(np.float32).astype(np.float64)
    Y = rng.standard_normal((201, 2)).astype(np.float32).astype(np.float64)
    for path in (N.FWD_AUTO, N.FWD_ROWS, N.FWD_NO_AGEMM):
        m._engine.set_forward_path(path, chunk_rows)
        outs = m._engine.forward(X, f_out="all")["F"]
        _, cache = O.forward(p, X, keep=True)
        for l in range(3):
            assert rel_err(cpu(outs[l][0]), cache[l][2] @ p.W[l]) < 5e-5, (path, l)
        acc = PredictiveLSE(m._engine, X, Y)
        acc.add_sample()
        ll, rmse = acc.finalize()
        lp, se = O.eval_log_likelihood_and_se(p, X, Y)
        ref_ll, ref_rmse = O.predictive_summary(lp[None], se[None])
        assert abs(ll - ref_ll) < 1e-4 and abs(rmse - ref_rmse) < 1e-5 * max(1.0, ref_rmse)
    m._engine.set_forward_path(N.FWD_AUTO)


def test_wide_first_layer_full_bayes_grad(dev):
    """full_bayesian=True gradients of a model whose first layer is wide (d = 40): the backward reads
    the precomputed A_1 and the X tile for the hyper-parameter sums."""
    from dgprf import engine as E
    from likelihoods import Softmax
    from models.dgp import DGP_RF
    from test_gpu_full_bayes import group_err
    E.set_seed(52)
    kinds, n_rf, n_gp = ["RBF", "RBF"], [64, 48], [6, 4]
    m = DGP_RF(40, 4, n_hidden_layers=2, n_rf=n_rf, n_gp=n_gp, likelihood=Softmax(),
               kernel_type_list=kinds)
    p = O.Params(40, 4, n_rf, n_gp, kinds, "softmax", False,
                 z=[cpu(m.BNN.layers[2 * l].z) for l in range(2)], W=[cpu(w) for w in m.W_mcmc],
                 log_inv_ls=[cpu(k.log_inv_length_scale) for k in m.kernel_list])
    rng = np.random.default_rng(9)
    X = rng.uniform(-1, 1, (37, 40)).astype(np.float32).astype(np.float64)
    Y = rng.integers(0, 4, (37, 1)).astype(float)
    eng = m._engine
    G = eng.grad(X, Y, 5000, full_bayes=True)
    ref = O.grad_full(p, X, Y, 5000, O.Trainable(kernel=True, lik=False, mean=False))
    Gw = unpack(eng, G[:, :eng.layout.w_total])
    pl = eng.layout
    h = cpu(G[0, pl.w_total:])
    for l in range(2):
        assert rel_err(Gw[l], ref["W"][l]) < 2e-4, ("W", l)
        lis = h[pl.lis_off[l]:pl.lis_off[l] + pl.d[l]]
        assert group_err(lis, ref["log_inv_ls"][l]) < 5e-4, ("lis", l)
    assert group_err([h[0], h[1]], [ref["log_amp"][0], ref["log_amp"][1]]) < 5e-4


def test_resident_first_layer_projection_steps(dev):
    """Wide first layer (d = 100 > 32), W-only graph steps: with Engine.resident_a1 the dataset's
    X Omega_1 is computed once (dataset_a1, the 128x128 MFMA GEMM) and every step gathers its
    minibatch's rows of it instead of running the step's A_1 GEMM; 6 graph steps match the GEMM
    form to fp32 rounding (the two GEMMs sum K in different orders), replay deterministically, and
    after an in-place hyper-parameter update (layer 0's length scales) the projection is rebuilt
    so the two forms still agree."""
    from dgprf import engine as E
    from likelihoods import Softmax
    from models.dgp import DGP_RF
    mk = lambda: DGP_RF(100, 5, n_hidden_layers=2, n_rf=[256, 128], n_gp=[10, 5],
                        likelihood=Softmax(), kernel_type_list=["RBF", "RBF"])
    models = []
    for _ in range(3):
        E.set_seed(54)
        models.append(mk())
    a, b, c = models
    b._engine.resident_a1 = False
    n = 2000
    X = torch.rand(n, 100, device=dev) * 2 - 1
    Y = torch.randint(0, 5, (n, 1), device=dev).float()
    for mm in models:
        mm.precond_update(None, n, precond_type="identity")
    for mm in (b, c):
        mm._engine.mom.copy_(a._engine.mom)
    run = dict(batch_size=96, lr=0.02, momentum_decay=0.9, steps_per_graph=3, perm_seed=2)
    for rnd in range(2):
        for mm in models:
            mm.run_sgmcmc(X, Y, n, 6, **run)
        torch.cuda.synchronize()
        assert a._engine._a1_cache and not b._engine._a1_cache
        scale = float(b._engine.theta.abs().max())
        assert float((a._engine.theta - b._engine.theta).abs().max()) <= 2e-5 * scale, rnd
        assert torch.equal(a._engine.theta, c._engine.theta), rnd  # deterministic replays
        with torch.no_grad():  # MCEM-style in-place update: Omega_1 and the projection rebuild
            for mm in models:
                mm.kernel_list[0].log_inv_length_scale.sub_(0.1)
    buf = next(iter(a._engine._a1_cache.values())).buf
    ref = X.double() @ a._engine.omega_view(0).double()
    assert float((buf[:n].double() - ref).abs().max()) <= 2e-5 * float(ref.abs().max())
    assert torch.all(buf[n:] == 0)


def test_wide_first_layer_two_chains_two_k_parts(dev):
    """C = 2 chains with a wide first layer (d = 100 > 32) at B = 96: the step's A_1 GEMM in two K
    parts (agemm.hip: blockIdx.y = chain x 2 + part, per-chain slab strides) feeding the layer-0
    forward / backward, which add slab 0 + slab 1 — each chain's gradient against the oracle with
    that chain's W, and chain 0 of 2-chain graph steps bitwise equal to a 1-chain engine."""
    from dgprf import engine as E
    from likelihoods import Softmax
    from models.dgp import DGP_RF
    E.set_seed(53)
    kinds, n_rf, n_gp = ["RBF", "RBF"], [256, 128], [10, 5]
    m = DGP_RF(100, 5, n_hidden_layers=2, n_rf=n_rf, n_gp=n_gp, likelihood=Softmax(),
               kernel_type_list=kinds)
    one = m._engine
    two = E.Engine(one.spec, 2, seed=one.seed)
    two.z.copy_(one.z)
    two.hyp.copy_(one.hyp)
    two.theta[0].copy_(one.theta[0])
    E.normal(None, 4, out=two.theta[1])
    assert two.layout.a0_off >= 0
    rng = np.random.default_rng(10)
    X = rng.uniform(-1, 1, (96, 100)).astype(np.float32).astype(np.float64)
    Y = rng.integers(0, 5, (96, 1)).astype(float)
    two.build_omega()
    G = two.grad(X, Y, 5000)
    for c in range(2):
        W = [cpu(two.theta[c, two.layout.w_off[l]:two.layout.w_off[l] + two.layout.P[l] * n_gp[l]])
             .reshape(two.layout.P[l], n_gp[l]) for l in range(2)]
        p = O.Params(100, 5, n_rf, n_gp, kinds, "softmax", False,
                     z=[cpu(m.BNN.layers[2 * l].z) for l in range(2)], W=W,
                     log_inv_ls=[cpu(k.log_inv_length_scale) for k in m.kernel_list])
        ref = O.grad_W(p, X, Y, 5000)
        got = unpack(two, G, chain=c)
        for l in range(2):
            assert rel_err(got[l], ref[l]) < 2e-4, (c, l)
    n = 960
    Xd = torch.rand(n, 100, device=dev) * 2 - 1
    Yd = torch.randint(0, 5, (n, 1), device=dev).float()
    for e in (one, two):
        e.mom.zero_()
        e.build_omega()
        e.graph(Xd, Yd, 96, n, 0.02, 0.9, 1.0, 5).launch()
    assert torch.equal(one.theta[0], two.theta[0])
    assert torch.isfinite(two.theta).all() and not torch.equal(two.theta[0], two.theta[1])


@pytest.mark.parametrize("n,d,ldx,R", [(200, 784, 784, 4096), (1024, 784, 784, 4096),
                                       (1025, 784, 784, 4096), (10_000, 784, 784, 4096),
                                       (77, 30, 33, 500), (1500, 36, 40, 1000)])
def test_rf_project_agemm_tiles(dev, n, d, ldx, R):
    """A = X Omega (layers/rf_layers.py:42) through dgprf_rf_project, the hand-written MFMA GEMM of
    the wide first layer, against a float64 matmul to 2e-5 of the output scale: config 4's first
    layer (d 784, R 4096) at the step's 200 rows and at 1,024 rows (64 x 64 tiles, K whole: the
    step itself runs them in two K parts, summed by its layer-0 kernels and covered by the config-4
    step parity tests), and past the switch at 1,025 and 10,000 rows (128 x 128 tiles, the
    benchmarked predictive chunk); a strided
    X (ldx > d) with d % 4 == 0 at 1,500 rows (128 x 128, ragged in every dimension); d = 30 (the
    LDS-tiled fallback kernel, rows written up to n only)."""
    from dgprf import engine as E
    from dgprf.engine import ModelSpec
    from dgprf import _native as N
    rng = np.random.default_rng(n + d)
    Xs = rng.uniform(-0.5, 0.5, (n, ldx)).astype(np.float32)
    om = (rng.standard_normal((d, R)) / np.sqrt(d)).astype(np.float32)
    eng = E.Engine(ModelSpec(4, 1, [N.RBF], [8], [1]))
    guard = torch.full((n + 40, R), 7.0, device=dev)  # rows past n must stay untouched
    A = eng.rf_project(torch.as_tensor(Xs, device=dev), torch.as_tensor(om, device=dev),
                       out=guard[:n])
    torch.cuda.synchronize()
    ref = Xs[:, :d].astype(np.float64) @ om.astype(np.float64)
    got = cpu(A)
    assert np.max(np.abs(got - ref)) < 2e-5 * np.max(np.abs(ref)), (n, d, R)
    assert torch.all(guard[n:] == 7.0)


def test_config4_predictive_rows_agemm_128(dev):
    """Config 4's full model (784-wide first layer, 4 x RBF n_rf 4096, softmax) scored on a ragged
    2,049-row test set in one A_1 chunk: the predictive path past 1,024 rows, whose A_1 GEMM runs
    the 128 x 128 tile instance (the benchmarked 10,000-row path's kernel); per-row log p against
    the float64 oracle (models/classification_model.py:49-60)."""
    c = CONFIGS[4]
    m, p = _model(c, 34)
    Xt, Yt = _data(c, 2049, 204)
    lp = cpu(m._engine.forward(Xt, Yt, logp=True)["logp"][0])
    ref = O.log_prob(p, O.forward(p, Xt), Yt)
    assert np.max(np.abs(lp - ref)) < 2e-5 * max(1.0, np.max(np.abs(ref)))


# ------------------------------------------------------------------ config 4's benchmarked step
# path: the resident X Omega_1 of the whole training set (Engine.dataset_a1) gathered per step in
# ceil(4096 / 1024) = 4 parts per row (gather_a1_part), read by the 8-wave layer-0 kernels
def _config4_resident_grad(eng, Xd, Yd, idx, N_, a1):
    """dU/dW [C, w_total] of the INDEXED minibatch idx [C, B] through the C-ABI dgprf_potential_grad
    (k_gather's resident-A_1 blocks for the rows, then the step's forward / backward) — with the
    dataset's resident projection a1, or the per-step A_1 GEMM when a1 is None."""
    import ctypes
    from dgprf import _native as N
    from dgprf.engine import ptr, stream
    B = idx.shape[1]
    pl, ws = eng.plan_ws(B)
    G = torch.zeros(eng.C, pl.w_total, device=Xd.device)
    ch = eng.chain_struct(ws)
    it = torch.as_tensor(idx, dtype=torch.int32, device=Xd.device).contiguous()
    bt = eng.batch_struct(Xd, Yd, N.BATCH_INDEXED, idx=it)
    bt.A1 = None if a1 is None else a1.data_ptr()
    N.call("dgprf_potential_grad", ctypes.byref(pl), ctypes.byref(ch), ctypes.byref(bt),
           float(N_), 0, ptr(G), stream())
    torch.cuda.synchronize()
    return G


def _config4_data(dev, n, seed):
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    X = torch.rand(n, 784, device=dev, generator=g) - 0.5  # normalize_MNIST range
    Y = torch.randint(0, 10, (n, 1), device=dev, generator=g).float()
    return X, Y


@pytest.mark.parametrize("C", [1, 4])
def test_config4_resident_a1_grad_vs_oracle(dev, C):
    """Config 4's full model (784 -> 4 x RBF n_rf 4096, g [30,30,30,10], softmax) at its benchmarked
    B = 200 over N = 60,000 rows: the gradient of an INDEXED minibatch whose first-layer rows are
    gathered from the resident X Omega_1 (4 gather parts of 1,024 features per row) against the
    float64 oracle (layers/rf_layers.py:42; models/dgp.py:194-198) for chain 0 and the last chain,
    and against the same step with the per-step A_1 GEMM; C = 4 chains sharing one hyper-parameter
    set (dataset_a1 serves them all) with their own rows and W."""
    import copy
    from dgprf import engine as E
    c = CONFIGS[4]
    m, p = _model(c, 70 + C)
    one = m._engine
    eng = one if C == 1 else E.Engine(one.spec, C, seed=one.seed)
    if C > 1:
        assert not eng.per_chain_hyp
        eng.z.copy_(one.z)
        eng.hyp.copy_(one.hyp)
        scale = 1.0 + 0.05 * torch.arange(C, device=dev, dtype=torch.float32)[:, None]
        eng.theta.copy_(one.theta[:1] * scale)
    eng.build_omega()
    n, B, N_ = 60_000, 200, 60_000
    Xd, Yd = _config4_data(dev, n, 404)
    a1 = eng.dataset_a1(Xd)
    assert a1 is not None and eng.layout.a0_off >= 0 and (eng.layout.n_rf[0] + 1023) // 1024 == 4
    rng = np.random.default_rng(405 + C)
    idx = np.stack([rng.choice(n, B, replace=False) for _ in range(C)]).astype(np.int32)
    G = _config4_resident_grad(eng, Xd, Yd, idx, N_, a1)
    Gg = _config4_resident_grad(eng, Xd, Yd, idx, N_, None)  # the per-step GEMM form
    assert torch.isfinite(G).all() and float(G.abs().max()) > 0
    for chain in range(C):
        for l, (x, y) in enumerate(zip(unpack(eng, G, chain), unpack(eng, Gg, chain))):
            assert rel_err(x, y) < 2e-5, ("resident vs GEMM", chain, l)
    Xh, Yh = cpu(Xd), cpu(Yd)
    for chain in sorted({0, C - 1}):
        pc = copy.copy(p)
        s = np.float64(np.float32(1.0 + 0.05 * chain))
        pc.W = [w * s for w in p.W]
        ref = O.grad_W(pc, Xh[idx[chain]], Yh[idx[chain]], N_)
        got = unpack(eng, G, chain=chain)
        for l in range(4):
            assert rel_err(got[l], ref[l]) < 2e-4, (C, chain, l)


def test_config4_resident_a1_graph_steps(dev):
    """Config 4's benchmarked step path as the bench runs it: W-only graph replays (2 x 5 steps, the
    first step of each replay gathering its A_1 rows in k_gather, the next ones in the update
    kernel's gather blocks) at B = 200 over N = 60,000 rows with the resident projection, against
    the same 10 steps with the per-step A_1 GEMM from the same state: theta within 2e-5 of its
    scale, and a third model replaying the resident path bit-identically."""
    from dgprf import engine as E
    c = CONFIGS[4]
    models = []
    for _ in range(3):
        m, _ = _model(c, 77)
        models.append(m)
    a, b, r = models
    b._engine.resident_a1 = False
    n = 60_000
    X, Y = _config4_data(dev, n, 406)
    for mm in models:
        E.set_seed(78)
        mm.precond_update(None, n, precond_type="identity")
    for mm in (b, r):
        mm._engine.mom.copy_(a._engine.mom)
        mm._engine.theta.copy_(a._engine.theta)
    run = dict(batch_size=200, lr=0.01, momentum_decay=0.9, steps_per_graph=5, perm_seed=9)
    for mm in models:
        mm.run_sgmcmc(X, Y, n, 10, **run)
    torch.cuda.synchronize()
    assert a._engine._a1_cache and not b._engine._a1_cache
    ta, tb = a._engine.theta, b._engine.theta
    assert torch.isfinite(ta).all()
    assert float((ta - tb).abs().max()) <= 2e-5 * float(tb.abs().max())
    assert torch.equal(ta, r._engine.theta)


# ------------------------------------------------------------------ resident projection cache
def test_dataset_a1_same_address_new_dataset(dev):
    """Two same-shape test sets created one after the other AT THE SAME ADDRESS with the same
    version count (what the caching allocator produces when the first set is freed and the second
    takes its block): each is scored against its own projection — equal to the GEMM path — and a
    freed dataset's entry leaves the cache.  The second set is built on the first one's storage
    explicitly (a fresh tensor object, its own version counter), so the case does not depend on
    the allocator's choices."""
    import gc
    from dgprf import engine as E
    from dgprf.predictive import PredictiveLSE
    from likelihoods import Softmax
    from models.dgp import DGP_RF
    E.set_seed(81)
    m = DGP_RF(100, 5, n_hidden_layers=2, n_rf=[256, 128], n_gp=[10, 5], likelihood=Softmax(),
               kernel_type_list=["RBF", "RBF"])
    eng = m._engine
    st = torch.empty(3000 * 100, device=dev).untyped_storage()
    Yt = torch.randint(0, 5, (3000, 1), device=dev).float()
    seen = []
    for seed in (1, 2):
        Xt = torch.empty(0, device=dev).set_(st, 0, (3000, 100))
        Xt.uniform_(-1 + 0.1 * seed, 1 + 0.1 * seed)
        seen.append((Xt.data_ptr(), tuple(Xt.shape), Xt._version))
        acc = PredictiveLSE(eng, Xt, Yt)
        acc.add_sample()
        ll, _ = acc.finalize()
        eng.resident_a1 = False
        ref = PredictiveLSE(eng, Xt, Yt)
        ref.add_sample()
        ll_ref, _ = ref.finalize()
        eng.resident_a1 = True
        assert abs(ll - ll_ref) < 1e-5 * max(1.0, abs(ll_ref)), seed
        assert len(eng._a1_cache) == 1
        del acc, ref, Xt
        gc.collect()
        assert not eng._a1_cache  # the finaliser dropped the freed dataset's projection
    # the old (address, shape, version) key could not tell the two sets apart
    assert seen[0] == seen[1], seen


def test_full_bayes_graph_replay_invalidates_projection(dev):
    """Full-Bayes graphs taken from sgmcmc_graphs and launched directly rewrite hyp / Omega_1 on the
    device at every replay: each launch advances hyper_epoch, so dataset_a1 afterwards is the
    projection of the CURRENT Omega_1, not of the one before the replays."""
    from dgprf import engine as E
    from likelihoods import Softmax
    from models.dgp import DGP_RF
    E.set_seed(82)
    m = DGP_RF(100, 5, n_hidden_layers=2, n_rf=[256, 128], n_gp=[10, 5], likelihood=Softmax(),
               kernel_type_list=["RBF", "RBF"])
    eng = m._engine
    n = 2000
    X = torch.rand(n, 100, device=dev) * 2 - 1
    Y = torch.randint(0, 5, (n, 1), device=dev).float()
    m.precond_update(None, n, precond_type="identity", full_bayesian=True)
    Xt = torch.rand(500, 100, device=dev) * 2 - 1
    plan = m.sgmcmc_graphs(X, Y, n, 20, batch_size=100, lr=0.05, momentum_decay=0.9,
                           steps_per_graph=10, full_bayesian=True)
    before = eng.dataset_a1(Xt).clone()
    ep = eng.hyper_epoch
    for g, reps in plan:
        for _ in range(reps):
            g.launch()
    assert eng.hyper_epoch == ep + 2
    now = eng.dataset_a1(Xt)
    ref = Xt.double() @ eng.omega_view(0).double()
    assert float((now[:500].double() - ref).abs().max()) <= 2e-5 * float(ref.abs().max())
    assert not torch.equal(now[:500], before[:500])  # Omega_1 did move


# ------------------------------------------------------------------ folded output layer
@pytest.mark.parametrize("kinds,n_rf,n_gp,D,B", [
    (["RBF"] * 3, [1024] * 3, [8, 8, 1], 8, 200),   # config 2 at its benchmarked B
    (["RBF"] * 3, [1024] * 3, [8, 8, 1], 8, 19),    # one ragged row tile
    (["RBF", "ARC"], [512, 512], [6, 1], 5, 77),    # ARC output layer (relu features)
    (["RBF"], [256], [1], 12, 50),                  # one layer: the folded layer reads X itself
])
def test_folded_output_layer_grad_and_step(dev, kinds, n_rf, n_gp, D, B):
    """plan.fold_out (step_fold_out): the output layer's forward is not launched; every backward
    workgroup of layer L recomputes its rows of F_L from the staged W_L / Omega_L.  Gradients of
    every layer against the float64 oracle, one injected-noise SGHMC step against the oracle's
    update, and the same gradient from a 4-chain engine (fold off: the forward launch and its 16
    slice partials) to fp32 rounding of the other summation order."""
    from dgprf import engine as E
    c = dict(kinds=kinds, n_rf=n_rf, n_gp=n_gp, D=D, lik="gaussian")
    m, p = _model(c, 90 + B)
    eng = m._engine
    L = len(kinds)
    pl, _ = eng.plan_ws(B)
    assert pl.fold_out == 1
    X, Y = _data(c, B, 91 + B)
    N_ = 50_000
    G = eng.grad(X, Y, N_)
    ref = O.grad_W(p, X, Y, N_)
    for l in range(L):
        assert rel_err(unpack(eng, G)[l], ref[l]) < 1e-4, ("grad", l)
    four = E.Engine(eng.spec, 4, seed=eng.seed)
    assert four.plan_ws(B)[0].fold_out == 0
    four.z.copy_(eng.z)
    four.hyp.copy_(eng.hyp)
    four.theta.copy_(eng.theta.expand(4, -1))
    four.lik_log_var_source = eng.lik_log_var_source
    four.build_omega()
    G4 = four.grad(X, Y, N_)
    for l in range(L):
        assert rel_err(unpack(four, G4)[l], unpack(eng, G)[l]) < 2e-5, ("4 chains", l)
    rng = np.random.default_rng(B)
    m.precond_update(None, N_, precond_type="identity")
    m0 = [cpu(eng.mom_view(l)).astype(np.float64) for l in range(L)]
    xi = [rng.standard_normal(w.shape) for w in p.W]
    eng.step(X, Y, N_, 0.01, 0.9, 1.0, xi=pack(eng, xi))
    O.sgmcmc_step(p, m0, X, Y, N_, 0.01, 0.9, 1.0, [1.0] * L, xi)
    for l in range(L):
        assert rel_err(cpu(eng.W_view(l)), p.W[l]) < 2e-5, ("step", l)

