"""full_bayesian=True on the HIP path (models/dgp.py:175-181, 199-216) against the CPU oracle.

The oracle's hyper-parameter gradients are pinned against torch autograd
(tests/test_oracle_autograd.py::test_full_bayes_grad_matches_autograd).  Tolerances (fp32 device vs
float64 oracle): W gradients 1e-4 of their scale, hyper-parameter gradients 5e-4 of the scale of
their group (they are sums over every row and feature), one update 1e-5 / 1e-4 (moments);
graph replays vs eager steps bit-exact.
"""
import numpy as np
import pytest
import torch

from oracle import dgp_oracle as O
from test_gpu_parity import (cpu, dev, model_from_fixture, oracle_params, pack,  # noqa: F401
                             rel_err, unpack)

pytestmark = pytest.mark.gpu

CASES = ["rbf2_gauss", "arc_rbf_softmax_cat", "mixed5", "wide_g"]


def trainable(g, eng):
    return O.Trainable(kernel=True, lik=int(g["dims"][3]) == 0, mean=True,
                       ard=[bool(eng.spec.ard[l]) for l in range(eng.L)])


def close(a, b, tol):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b))) <= tol * (1.0 + float(np.max(np.abs(b))))


def hyper_of(eng, vec):
    """Split a [hyp_total] vector (hyp layout) into the oracle's per-variable structure."""
    pl = eng.layout
    v = cpu(vec) if torch.is_tensor(vec) else vec
    L = eng.L
    nl = lambda l: pl.d[l] if eng.spec.ard[l] else 1
    return {"log_amp": [v[l] for l in range(L)],
            "log_inv_ls": [v[pl.lis_off[l]:pl.lis_off[l] + nl(l)] for l in range(L)],
            "mean": [v[pl.mean_off[l]:pl.mean_off[l] + pl.d[l]] for l in range(L)],
            "lik_log_var": v[L]}


def hyper_to(eng, per_var):
    """Inverse of hyper_of -> float32 [1, hyp_total] device tensor."""
    pl = eng.layout
    t = np.zeros(pl.hyp_total, np.float32)
    for l in range(eng.L):
        t[l] = per_var["log_amp"][l]
        t[pl.lis_off[l]:pl.lis_off[l] + pl.d[l]] = per_var["log_inv_ls"][l]
        t[pl.mean_off[l]:pl.mean_off[l] + pl.d[l]] = per_var["mean"][l]
    t[eng.L] = per_var["lik_log_var"]
    return torch.as_tensor(t)[None].to(eng.dev)


def group_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / (np.max(np.abs(b)) + 1e-30))


@pytest.mark.parametrize("name", CASES)
def test_full_bayes_potential_grad(dev, golden, name):
    g = golden(name)
    m = model_from_fixture(g)
    eng = m._engine
    N_ = int(g["dims"][5])
    G = eng.grad(g["X"], g["Y"], N_, full_bayes=True)
    assert G.shape == (1, eng.layout.w_total + eng.layout.hyp_total)
    ref = O.grad_full(oracle_params(g), g["X"], g["Y"], N_, trainable(g, eng))
    Gw = unpack(eng, G[:, :eng.layout.w_total])
    Gh = hyper_of(eng, G[0, eng.layout.w_total:])
    for l in range(m.n_hidden_layers):
        assert rel_err(Gw[l], ref["W"][l]) < 1e-4, (name, "W", l)
        for key in ("log_inv_ls", "mean"):
            assert group_err(Gh[key][l], ref[key][l]) < 5e-4, (name, key, l)
    # log_amp: compare the per-layer scalars as one group (their common scale)
    assert group_err([Gh["log_amp"][l] for l in range(m.n_hidden_layers)],
                     [ref["log_amp"][l] for l in range(m.n_hidden_layers)]) < 5e-4
    if ref["lik_log_var"] is not None:
        assert abs(Gh["lik_log_var"] - ref["lik_log_var"]) < 5e-4 * (abs(ref["lik_log_var"]) + 1.0)
    # the W part agrees with the W-only gradient (another kernel instantiation: fp32 order only)
    assert rel_err(cpu(G[:, :eng.layout.w_total]), cpu(eng.grad(g["X"], g["Y"], N_))) < 1e-6


@pytest.mark.parametrize("name", ["rbf2_gauss", "arc_rbf_softmax_cat", "mixed5"])
@pytest.mark.parametrize("resample", [False, True])
def test_full_bayes_step_injected_noise(dev, golden, name, resample):
    g = golden(name)
    m = model_from_fixture(g)
    eng = m._engine
    L = m.n_hidden_layers
    tr = trainable(g, eng)
    lr, beta, T, N_ = g["step_scalars"]
    rng = np.random.default_rng(17)
    p = oracle_params(g)
    keys = O.full_groups(p, tr)
    mom = {k: rng.standard_normal(np.shape(O.get_var(p, k, tr))) for k in keys}
    xi = {k: rng.standard_normal(np.shape(O.get_var(p, k, tr))) for k in keys}
    xr = {k: rng.standard_normal(np.shape(O.get_var(p, k, tr))) for k in keys} if resample else None
    Mv = {k: float(rng.uniform(0.5, 2.0)) for k in keys}
    # device state: W momenta / masses, hyper momenta / masses, injected noise
    pick = lambda d_, nm, l: d_.get((nm, l), None)
    with torch.no_grad():
        for l in range(L):
            eng.mom_view(l).copy_(torch.as_tensor(mom[("W", l)]))
            eng.mass[0, l] = Mv[("W", l)]
            eng.hmass[0, l] = Mv[("log_amp", l)]
            eng.hmass[0, 8 + l] = Mv[("log_inv_ls", l)]
            eng.hmass[0, 16 + l] = Mv[("mean", l)]
        if ("lik_log_var", None) in Mv:
            eng.hmass[0, 24] = Mv[("lik_log_var", None)]

    def hyp_tensor(src):
        per = {"log_amp": [], "log_inv_ls": [], "mean": []}
        for l in range(L):
            for nm in per:
                v = pick(src, nm, l)
                per[nm].append(np.zeros(np.shape(O.get_var(p, (nm, l), tr))) if v is None else v)
        per["lik_log_var"] = src.get(("lik_log_var", None), 0.0)
        return hyper_to(eng, per)

    eng.hmom.copy_(hyp_tensor(mom))
    eng.moments_ready = eng.hyper_moments_ready = True
    xiw = pack(eng, [xi[("W", l)] for l in range(L)])
    xrw = pack(eng, [xr[("W", l)] for l in range(L)]) if resample else None
    xih = hyp_tensor(xi)
    xrh = hyp_tensor(xr) if resample else None
    eng.step(g["X"], g["Y"], N_, lr, beta, T, resample=resample, xi=xiw, xi_resample=xrw,
             full_bayes=True, xi_hyp=xih, xi_hyp_resample=xrh)
    new_m = O.sgmcmc_step_full(p, mom, g["X"], g["Y"], N_, lr, beta, T, Mv, xi, tr, xr)
    for l in range(L):
        assert rel_err(cpu(eng.W_view(l)), p.W[l]) < 1e-5, ("W", l)
        assert rel_err(cpu(eng.mom_view(l)), new_m[("W", l)]) < 1e-4, ("mW", l)
    h = hyper_of(eng, eng.hyp_chain(0))
    hm = hyper_of(eng, eng.hmom[0])
    for l in range(L):
        hv = cpu(eng.hyp_chain(0))
        assert close(h["log_amp"][l], p.log_amp[l], 1e-5)
        # every length-scale slot holds the sampled value (scalar ARD: broadcast)
        o = eng.layout.lis_off[l]
        assert close(hv[o:o + p.d[l]], p.log_inv_ls[l], 1e-5), ("lis", l)
        assert close(h["mean"][l], p.mean[l], 1e-5)
        for nm in ("log_amp", "log_inv_ls", "mean"):
            assert group_err(hm[nm][l], new_m[(nm, l)]) < 1e-4, (nm, l)
        # Omega and c were rebuilt on the device from the new hyper-parameters
        assert rel_err(cpu(eng.omega_view(l)), O.omega(p, l)) < 1e-5
        assert abs(float(cpu(eng.c_view(l))[0]) - O.amp_scale(p, l)) < 1e-5 * O.amp_scale(p, l)
    if tr.lik and p.likelihood == "gaussian":
        assert close(h["lik_log_var"], p.lik_log_var, 1e-5)
        assert group_err(hm["lik_log_var"], new_m[("lik_log_var", None)]) < 1e-4
        assert abs(float(cpu(eng.der[8:9])[0]) - np.exp(p.lik_log_var)) < 1e-5 * np.exp(p.lik_log_var)
        # the likelihood object sees the sampled value (bound to its engine slot)
        assert abs(float(cpu(m.likelihood.lik_log_var)) - p.lik_log_var) < 1e-5


def test_full_bayes_graph_equals_eager_steps(dev):
    from likelihoods import Gaussian
    from models.regression_model import RegressionDGP
    from dgprf import engine as E
    mk = lambda: RegressionDGP(4, 1, n_hidden_layers=2, n_rf=40, n_gp=[3, 1],
                               likelihood=Gaussian(), set_nonzero_mean=True)
    E.set_seed(21)
    a = mk()
    E.set_seed(21)
    b = mk()
    n, B = 640, 64
    X = torch.randn(n, 4, device=dev)
    Y = torch.randn(n, 1, device=dev)
    for mm in (a, b):
        mm.precond_update(None, n, precond_type="identity", full_bayesian=True)
    b._engine.mom.copy_(a._engine.mom)
    b._engine.hmom.copy_(a._engine.hmom)
    a.run_sgmcmc(X, Y, n, 16, batch_size=B, lr=0.01, momentum_decay=0.9, steps_per_graph=8,
                 perm_seed=3, full_bayesian=True)
    for _ in range(16):
        b._engine.step(X, Y, n, 0.01, 0.9, 1.0, batch_size=B, mode=2, perm_seed=3,
                       full_bayes=True)
    ea, eb = a._engine, b._engine
    assert int(ea.step_ctr) == 16 == int(eb.step_ctr)
    for t in ("theta", "mom", "hyp", "hmom", "omega", "der"):
        assert torch.equal(getattr(ea, t), getattr(eb, t)), t
    # the hyper-parameters moved
    assert not torch.equal(ea.hyp, mk()._engine.hyp)


def test_full_bayes_precond_rmsprop_masses(dev, golden):
    from likelihoods import Gaussian
    from models.regression_model import RegressionDGP
    from test_gpu_parity import load_params
    g = golden("precond")
    m = RegressionDGP(2, 1, n_hidden_layers=2, n_rf=[16, 24], n_gp=[3, 1],
                      likelihood=Gaussian(variance=float(np.exp(g["lik_log_var"]))),
                      set_nonzero_mean=True)
    g2 = dict(g)
    g2["kinds"] = np.array([0, 0])
    load_params(m, g2)
    g2["dims"] = np.array([2, 1, 0, 0])
    g2["n_rf"], g2["n_gp"] = np.array([16, 24]), np.array([3, 1])
    p = oracle_params(g2)
    tr = O.Trainable(kernel=True, lik=True, mean=True)
    K = 4
    ds = [(g["Xs"][k], g["Ys"][k]) for k in range(K)]
    m.precond_update(None, int(g["N"]), precond_type="identity", full_bayesian=True)
    eng = m._engine
    m0, h0 = cpu(eng.mom).copy(), cpu(eng.hmom).copy()
    m.precond_update(ds, int(g["N"]), K_batches=K, full_bayesian=True)
    # oracle: Welford over K full-Bayes gradients per variable, masses normalised by the minimum
    grads = [O.grad_full(p, ds[k][0], ds[k][1], int(g["N"]), tr) for k in range(K)]
    masses = {}
    for key in O.full_groups(p, tr):
        nm, l = key
        gs = [np.asarray(gr[nm] if l is None else gr[nm][l], np.float64) for gr in grads]
        mean, m2 = np.zeros_like(gs[0]), np.zeros_like(gs[0])
        for k in range(K):
            mean, m2 = O.welford(mean, m2, gs[k], k + 1)
        masses[key] = O.mass_estimate(mean, m2, K, False)
    mmin = min(masses.values())
    pl = eng.layout
    for l in range(2):
        assert abs(float(cpu(eng.mass)[0, l]) - masses[("W", l)] / mmin) < 1e-4 * masses[("W", l)] / mmin
        for nm, slot in (("log_amp", l), ("log_inv_ls", 8 + l), ("mean", 16 + l)):
            ref = masses[(nm, l)] / mmin
            assert abs(float(cpu(eng.hmass)[0, slot]) - ref) < 2e-4 * ref, (nm, l)
    ref = masses[("lik_log_var", None)] / mmin
    assert abs(float(cpu(eng.hmass)[0, 24]) - ref) < 2e-4 * ref
    # hyper momenta rescaled by sqrt(M) (rsqrt(1) * moments before)
    M_amp0 = float(cpu(eng.hmass)[0, 0])
    assert abs(float(cpu(eng.hmom)[0, 0]) - np.sqrt(M_amp0) * h0[0, 0]) < 1e-5 * (1 + abs(h0[0, 0]))
    o = pl.lis_off[1]
    M_l1 = float(cpu(eng.hmass)[0, 9])
    assert rel_err(cpu(eng.hmom)[0, o:o + pl.d[1]], np.sqrt(M_l1) * h0[0, o:o + pl.d[1]]) < 1e-5


# ----------------------------------------------------------------------------- engine level
def load_chain(eng, p, c):
    """Write oracle Params p into chain c of an Engine (z is shared by all chains)."""
    pl = eng.layout
    with torch.no_grad():
        for l in range(eng.L):
            eng.z_view(l).copy_(torch.as_tensor(p.z[l]))
            eng.W_view(l, c).copy_(torch.as_tensor(p.W[l]))
        h = eng.hyp_chain(c)
        for l in range(eng.L):
            h[l] = float(p.log_amp[l])
            h[pl.lis_off[l]:pl.lis_off[l] + pl.d[l]] = torch.as_tensor(p.log_inv_ls[l])
            h[pl.mean_off[l]:pl.mean_off[l] + pl.d[l]] = torch.as_tensor(p.mean[l])
        h[eng.L] = float(p.lik_log_var)


def random_params(rng, spec_args, ard):
    d_in, d_out, kinds, n_rf, n_gp, cat, lik = spec_args
    d = O.layer_widths(d_in, n_gp, cat)
    L = len(kinds)
    lis = [O.init_log_inv_ls(d[l]) + (0.2 * rng.standard_normal(d[l]) if ard[l] else 0.0)
           for l in range(L)]
    return O.Params(d_in, d_out, n_rf, n_gp, kinds, lik, cat, rng=rng,
                    log_amp=[0.2 * rng.standard_normal() for _ in range(L)], log_inv_ls=lis,
                    mean=[0.2 * rng.standard_normal(d[l]) for l in range(L)],
                    lik_log_var=np.log(0.2) + 0.1 * rng.standard_normal())


ENGINE_CASES = [
    # d_in, d_out, kinds, n_rf, n_gp, cat, lik | ard | hyp flags
    ((3, 1, ["RBF", "ARC", "RBF"], [32, 48, 20], [4, 5, 1], False, "gaussian"), [0, 1, 0],
     ("kernel", "lik", "mean")),
    ((5, 3, ["ARC", "RBF"], [40, 24], [6, 3], True, "softmax"), [1, 0], ("kernel",)),
    ((2, 2, ["RBF", "RBF"], [16, 100], [3, 2], False, "gaussian"), [1, 1], ("mean", "lik")),
    ((20, 1, ["RBF"], [64], [1], False, "gaussian"), [0], ("kernel", "lik")),
]


def engine_for(spec_args, ard, flags, C=1):
    from dgprf import _native as N
    from dgprf import engine as E
    d_in, d_out, kinds, n_rf, n_gp, cat, lik = spec_args
    hf = (N.HYP_KERNEL if "kernel" in flags else 0) | (N.HYP_LIK if "lik" in flags else 0) | \
        (N.HYP_MEAN if "mean" in flags else 0)
    spec = E.ModelSpec(d_in, d_out, [N.RBF if k == "RBF" else N.ARC for k in kinds], n_rf, n_gp,
                       cat, N.LIK_GAUSSIAN if lik == "gaussian" else N.LIK_SOFTMAX, hf, ard)
    return E.Engine(spec, n_chains=C, per_chain_hyp=True)


def check_grad(eng, G, c, ref, tr):
    pl = eng.layout
    Gw = unpack(eng, G[:, :pl.w_total], chain=c)
    Gh = hyper_of(eng, G[c, pl.w_total:])
    for l in range(eng.L):
        assert rel_err(Gw[l], ref["W"][l]) < 1e-4, ("W", l)
        if tr.kernel:
            assert group_err(Gh["log_inv_ls"][l], ref["log_inv_ls"][l]) < 5e-4, ("lis", l)
        if tr.mean:
            assert group_err(Gh["mean"][l], ref["mean"][l]) < 5e-4, ("mean", l)
    if tr.kernel:
        assert group_err([Gh["log_amp"][l] for l in range(eng.L)],
                         [ref["log_amp"][l] for l in range(eng.L)]) < 5e-4
    if ref["lik_log_var"] is not None:
        assert abs(Gh["lik_log_var"] - ref["lik_log_var"]) < 5e-4 * (abs(ref["lik_log_var"]) + 1)
    # slots of groups that do not train carry zero gradient
    if not tr.kernel:
        assert all(Gh["log_amp"][l] == 0 for l in range(eng.L))
    if not tr.mean:
        assert all(np.all(Gh["mean"][l] == 0) for l in range(eng.L))


@pytest.mark.parametrize("case", range(len(ENGINE_CASES)))
def test_full_bayes_engine_grad_flags_and_scalar_lengthscale(dev, case):
    spec_args, ard, flags = ENGINE_CASES[case]
    rng = np.random.default_rng(100 + case)
    eng = engine_for(spec_args, ard, flags)
    p = random_params(rng, spec_args, ard)
    load_chain(eng, p, 0)
    B, N_ = 77, 5000
    X = rng.standard_normal((B, spec_args[0]))
    Y = rng.standard_normal((B, spec_args[1])) if spec_args[6] == "gaussian" else \
        rng.integers(0, spec_args[1], (B, 1)).astype(float)
    tr = O.Trainable(kernel="kernel" in flags, lik="lik" in flags, mean="mean" in flags,
                     ard=[bool(a) for a in ard])
    G = eng.grad(X, Y, N_, full_bayes=True)
    check_grad(eng, G, 0, O.grad_full(p, X, Y, N_, tr), tr)


@pytest.mark.parametrize("case,B", [(0, 600), (1, 600), (0, 2048)])
def test_full_bayes_row_group_grad(dev, case, B):
    """B = 600 (38 row tiles: row-group kernel) and B = 2048 (8 row tiles per group: row-wave
    kernel): the full-Bayes backward keeps the hyper-parameter partials per row group (<= 16 rows)
    like gW; every gradient against the oracle."""
    spec_args, ard, flags = ENGINE_CASES[case]
    rng = np.random.default_rng(300 + case)
    eng = engine_for(spec_args, ard, flags)
    p = random_params(rng, spec_args, ard)
    load_chain(eng, p, 0)
    N_ = 5000
    pl = eng.plan_ws(B)[0]
    n_rt = (B + 15) // 16
    assert pl.rt_per_group == -(-n_rt // 16) and pl.n_gw_rows <= 16 and pl.rg_full_bayes == 1
    X = rng.standard_normal((B, spec_args[0]))
    Y = rng.standard_normal((B, spec_args[1])) if spec_args[6] == "gaussian" else \
        rng.integers(0, spec_args[1], (B, 1)).astype(float)
    tr = O.Trainable(kernel="kernel" in flags, lik="lik" in flags, mean="mean" in flags,
                     ard=[bool(a) for a in ard])
    G = eng.grad(X, Y, N_, full_bayes=True)
    check_grad(eng, G, 0, O.grad_full(p, X, Y, N_, tr), tr)


@pytest.mark.parametrize("case", [0, 1])
def test_full_bayes_engine_step_scalar_lengthscale(dev, case):
    """One step with injected noise; scalar length scales stay broadcast over their d slots."""
    spec_args, ard, flags = ENGINE_CASES[case]
    rng = np.random.default_rng(200 + case)
    eng = engine_for(spec_args, ard, flags)
    p = random_params(rng, spec_args, ard)
    load_chain(eng, p, 0)
    tr = O.Trainable(kernel="kernel" in flags, lik="lik" in flags, mean="mean" in flags,
                     ard=[bool(a) for a in ard])
    B, N_, lr, beta, T = 50, 2000, 0.01, 0.9, 1.0
    X = rng.standard_normal((B, spec_args[0]))
    Y = rng.standard_normal((B, spec_args[1])) if spec_args[6] == "gaussian" else \
        rng.integers(0, spec_args[1], (B, 1)).astype(float)
    keys = O.full_groups(p, tr)
    shp = lambda k: np.shape(O.get_var(p, k, tr))
    mom = {k: rng.standard_normal(shp(k)) for k in keys}
    xi = {k: rng.standard_normal(shp(k)) for k in keys}
    Mv = {k: (1.0 if k[0] == "W" else float(rng.uniform(0.5, 2.0))) for k in keys}
    pl = eng.layout
    slot = {"log_amp": lambda l: (l, l), "log_inv_ls": lambda l: (8 + l, pl.lis_off[l]),
            "mean": lambda l: (16 + l, pl.mean_off[l]), "lik_log_var": lambda l: (24, eng.L)}
    hm = torch.zeros(1, pl.hyp_total)
    xh = torch.zeros(1, pl.hyp_total)
    with torch.no_grad():
        for k in keys:
            nm, l = k
            if nm == "W":
                eng.mom_view(l).copy_(torch.as_tensor(mom[k]))
                continue
            s, o = slot[nm](l)
            eng.hmass[0, s] = Mv[k]
            n = int(np.size(mom[k]))
            hm[0, o:o + n] = torch.as_tensor(np.reshape(mom[k], -1))
            xh[0, o:o + n] = torch.as_tensor(np.reshape(xi[k], -1))
        eng.hmom.copy_(hm)
    eng.moments_ready = eng.hyper_moments_ready = True
    xiw = pack(eng, [xi[("W", l)] for l in range(eng.L)])
    eng.step(X, Y, N_, lr, beta, T, xi=xiw, full_bayes=True, xi_hyp=xh.to(dev))
    new_m = O.sgmcmc_step_full(p, mom, X, Y, N_, lr, beta, T, Mv, xi, tr)
    h = cpu(eng.hyp_chain(0))
    hmv = cpu(eng.hmom[0])
    for l in range(eng.L):
        assert rel_err(cpu(eng.W_view(l)), p.W[l]) < 1e-5
        assert close(h[pl.lis_off[l]:pl.lis_off[l] + pl.d[l]], p.log_inv_ls[l], 1e-5), l
        assert close(h[pl.mean_off[l]:pl.mean_off[l] + pl.d[l]], p.mean[l], 1e-5), l
        assert close(h[l], p.log_amp[l], 1e-5)
        assert rel_err(cpu(eng.omega_view(l)), O.omega(p, l)) < 1e-5
        if ("log_inv_ls", l) in new_m:
            n = int(np.size(new_m[("log_inv_ls", l)]))
            o = pl.lis_off[l]
            assert group_err(hmv[o:o + n], new_m[("log_inv_ls", l)]) < 1e-4
    if ("lik_log_var", None) in new_m:
        assert close(h[eng.L], p.lik_log_var, 1e-5)


def test_full_bayes_per_chain_hyper_parameters(dev):
    """C chains, each with its own hyper-parameters / Omega (per_chain_hyp): every chain's
    gradient and forward match the oracle at that chain's state."""
    spec_args, ard, flags = ENGINE_CASES[0]
    C = 3
    rng = np.random.default_rng(300)
    eng = engine_for(spec_args, ard, flags, C=C)
    ps = [random_params(rng, spec_args, ard) for _ in range(C)]
    for c in range(1, C):
        ps[c].z = ps[0].z                       # z is shared by the chains
    for c in range(C):
        load_chain(eng, ps[c], c)
    tr = O.Trainable(kernel=True, lik=True, mean=True, ard=[bool(a) for a in ard])
    B, N_ = 64, 3000
    X = rng.standard_normal((B, spec_args[0]))
    Y = rng.standard_normal((B, 1))
    G = eng.grad(X, Y, N_, full_bayes=True)
    for c in range(C):
        check_grad(eng, G, c, O.grad_full(ps[c], X, Y, N_, tr), tr)
    # forward per chain uses that chain's Omega
    F = eng.forward(X, f_out=True)["F"][0]
    for c in range(C):
        assert rel_err(cpu(F[c]), O.forward(ps[c], X)) < 2e-5, c


@pytest.mark.parametrize("C", [4, 16])
def test_full_bayes_per_chain_wide_slices(dev, C):
    """Per-chain hyper-parameters with 4 / 16 chains, whose plans take wider feature slices
    (4 / 8 16-feature chunks per wave at n_rf = 1024): the full-Bayes gradient of the first and
    last chain matches the oracle at that chain's state."""
    spec_args = (3, 1, ["RBF", "ARC"], [1024, 512], [4, 1], False, "gaussian")
    ard, flags = [0, 1], ("kernel", "lik", "mean")
    rng = np.random.default_rng(310 + C)
    eng = engine_for(spec_args, ard, flags, C=C)
    assert eng.layout.cpw[0] == (8 if C >= 16 else 4)
    ps = [random_params(rng, spec_args, ard) for _ in range(C)]
    for c in range(1, C):
        ps[c].z = ps[0].z
    for c in range(C):
        load_chain(eng, ps[c], c)
    tr = O.Trainable(kernel=True, lik=True, mean=True, ard=[bool(a) for a in ard])
    B, N_ = 64, 3000
    X = rng.standard_normal((B, spec_args[0]))
    Y = rng.standard_normal((B, 1))
    G = eng.grad(X, Y, N_, full_bayes=True)
    for c in (0, C - 1):
        check_grad(eng, G, c, O.grad_full(ps[c], X, Y, N_, tr), tr)


def test_full_bayes_config4_shape_large_batch(dev):
    """full_bayesian=True at BASELINE config 4's model shape (784-wide first layer, 4 x RBF n_rf
    4096, g [30,30,30,10], softmax) with B = 600: the W-only row-group layout fits, the full-Bayes
    one does not (staged X + hyper sums > 160 KiB), so the engine takes the per-row-tile backward
    plan (plan.bwd_tiles) instead of failing with E_SHAPE.  Every gradient against the
    oracle (W: 2e-4 of the gradient scale, the K = 8,192 contractions of config 4)."""
    spec_args = (784, 10, ["RBF"] * 4, [4096] * 4, [30, 30, 30, 10], False, "softmax")
    ard = [1] * 4
    rng = np.random.default_rng(404)
    eng = engine_for(spec_args, ard, ("kernel",))
    p = random_params(rng, spec_args, ard)
    for l in range(4):
        p.mean[l] = np.zeros_like(p.mean[l])  # mean not trainable here: keep the default 0
    load_chain(eng, p, 0)
    B, N_ = 600, 60_000
    pw = eng.plan_ws(B)[0]
    assert pw.rt_per_group > 1 and pw.rg_full_bayes == 0
    pf = eng.plan_ws(B, full_bayes=True)[0]
    assert pf.rt_per_group == 1 and pf.bwd_tiles == 1 and pf.n_gw_rows == (B + 15) // 16
    X = rng.uniform(-0.5, 0.5, (B, 784))
    Y = rng.integers(0, 10, (B, 1)).astype(float)
    tr = O.Trainable(kernel=True, lik=False, mean=False, ard=[True] * 4)
    G = eng.grad(X, Y, N_, full_bayes=True)
    ref = O.grad_full(p, X, Y, N_, tr)
    pl = eng.layout
    Gw = unpack(eng, G[:, :pl.w_total])
    Gh = hyper_of(eng, G[0, pl.w_total:])
    for l in range(4):
        assert rel_err(Gw[l], ref["W"][l]) < 2e-4, ("W", l)
        assert group_err(Gh["log_inv_ls"][l], ref["log_inv_ls"][l]) < 5e-4, ("lis", l)
    assert group_err([Gh["log_amp"][l] for l in range(4)], [ref["log_amp"][l] for l in range(4)]) < 5e-4
    # the W part equals the W-only row-group gradient up to fp32 summation order
    assert rel_err(cpu(G[:, :pl.w_total]), cpu(eng.grad(X, Y, N_))) < 1e-5
