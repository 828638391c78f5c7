"""Posterior-predictive parity at BASELINE sizes: the HIP forward's online
log-sum-exp folded over samples, chains and ranks, against the float64 oracle's
experiments/utils_training.py:79-85 aggregation (oracle.predictive_summary) over the same samples.

Tolerances (north_star): |dLL| < 1e-4 absolute; RMSE relative < 1e-5; per-point LSE |d| < 1e-4.
The device path is the product one: hardware v_sin/v_cos after v_fract range reduction (the default
build), one tile-kernel launch per sample with grid.y = C chains, k_lse_finalize over `parts`
accumulator rows (chains x ranks).
"""
import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import dgp_oracle as O
from test_gpu_parity import cpu, dev  # noqa: F401

pytestmark = pytest.mark.gpu

CFG2 = dict(kinds=["RBF"] * 3, n_rf=[1024] * 3, n_gp=[8, 8, 1], D=8, variance=0.1)


def _build_config2():
    from likelihoods import Gaussian
    from models.regression_model import RegressionDGP
    return RegressionDGP(CFG2["D"], 1, n_hidden_layers=3, n_rf=CFG2["n_rf"], n_gp=CFG2["n_gp"],
                         likelihood=Gaussian(variance=CFG2["variance"]))


def _config2_model(seed):
    from dgprf import engine as E
    E.set_seed(seed)
    return _build_config2()


def _oracle_params(m, W):
    """Oracle parameters of model m's kernels / frequencies with the GP weights W (list per layer)."""
    L = m.n_hidden_layers
    return O.Params(CFG2["D"], 1, CFG2["n_rf"], CFG2["n_gp"], CFG2["kinds"], "gaussian", False,
                    z=[cpu(m.BNN.layers[2 * l].z) for l in range(L)], W=W,
                    log_amp=[cpu(k.log_amplitude) for k in m.kernel_list],
                    log_inv_ls=[cpu(k.log_inv_length_scale) for k in m.kernel_list],
                    lik_log_var=np.log(CFG2["variance"]))


def _unpack(eng, theta_row):
    pl = eng.layout
    return [np.asarray(theta_row[pl.w_off[l]:pl.w_off[l] + pl.P[l] * pl.n_gp[l]],
                       dtype=np.float64).reshape(pl.P[l], pl.n_gp[l]) for l in range(eng.L)]


def _oracle_lp_se(p, X, Y, chunk=10_000):
    """Per-point log p and se of one sample, the oracle forward in row chunks (bounded memory)."""
    lp, se = [], []
    for i in range(0, X.shape[0], chunk):
        a, b = O.eval_log_likelihood_and_se(p, X[i:i + chunk], Y[i:i + chunk])
        lp.append(a)
        se.append(b)
    return np.concatenate(lp), np.concatenate(se)


def _oracle_lse(lp, y_std=1.0):
    l = np.asarray(lp, np.float64) - np.log(y_std)
    mx = l.max(axis=0)
    return mx + np.log(np.exp(l - mx).sum(axis=0))


def test_predictive_ll_config2_70k_rows_4_samples(dev):
    """Config 2's model (3 x RBF, n_rf 1024, g [8,8,1]) scored on N_t = 70,001 rows (one round of
    resident tiles plus a ragged remainder) for S = 4 posterior samples drawn by graph-replayed
    SGHMC on device-resident data: LL within 1e-4 and RMSE within 1e-5 relative of the oracle over
    the same 4 samples, y_std = 1 and y_std = 1.7 (utils_training.py:63-64)."""
    from dgprf.data import regression_data
    from dgprf.predictive import PredictiveLSE
    n_train, n_test = 100_000, 70_001
    X, Y, a = regression_data(n_train, CFG2["D"], seed=0, device=dev)
    Xt, Yt, _ = regression_data(n_test, CFG2["D"], seed=1, device=dev, a=a)
    m = _config2_model(2)
    m.precond_update(None, n_train, precond_type="identity")
    acc = PredictiveLSE(m._engine, Xt, Yt)
    Ws = []
    for s in range(4):
        m.run_sgmcmc(X, Y, n_train, 40, batch_size=200, lr=0.01, momentum_decay=0.9,
                     steps_per_graph=20, perm_seed=3)
        acc.add_sample()
        Ws.append([cpu(w).astype(np.float64) for w in m.W_mcmc])
    Xh, Yh = cpu(Xt).astype(np.float64), cpu(Yt).astype(np.float64)
    lps, ses = zip(*[_oracle_lp_se(_oracle_params(m, W), Xh, Yh) for W in Ws])
    for y_std in (1.0, 1.7):
        ll, rmse = acc.finalize(y_std=y_std)
        ref_ll, ref_rmse = O.predictive_summary(np.stack(lps), np.stack(ses), y_std=y_std)
        assert abs(ll - ref_ll) < 1e-4, (y_std, ll, ref_ll)
        assert abs(rmse - ref_rmse) < 1e-5 * ref_rmse, (y_std, rmse, ref_rmse)


@pytest.mark.parametrize("C,S", [(1, 4), (2, 3)])
def test_predictive_two_samples_per_launch(dev, C, S):
    """PredictiveLSE.add_samples (dgprf::forward_samples): config 2's model scores two posterior
    samples per pass of the pair kernel — layer 0's A = X Omega_1 and cos / sin once for both, its
    F contraction on 16x16x4 MFMA tiles with the two samples' W side by side — and folds every
    sample into the chain's accumulators in sample order; an odd S ends with a one-sample pass.
    LL within 1e-4 and RMSE within 1e-5 relative of the oracle over the C x S samples, and the
    per-point LSE within 2e-5 of max(1, |LSE|) of the oracle's, as the same samples folded one
    launch at a time (add_sample) are."""
    from dgprf import _native as N
    from dgprf import engine as E
    from dgprf.data import regression_data
    from dgprf.predictive import PredictiveLSE
    n_test = 20_001
    Xt, Yt, _ = regression_data(n_test, CFG2["D"], seed=7, device=dev)
    m = _config2_model(11)
    eng = m._engine if C == 1 else _multi_chain_engine(m, C, seed=78)
    eng.build_omega()
    E.set_seed(12)
    thetas = torch.stack([E.normal((C, eng.layout.w_total), N.RNG_W) for _ in range(S)])
    pair = PredictiveLSE(eng, Xt, Yt)
    pair.add_samples(thetas, build=False)
    one = PredictiveLSE(eng, Xt, Yt)
    keep = eng.theta.clone()
    for s in range(S):
        eng.theta.copy_(thetas[s])
        one.add_sample(build=False)
    eng.theta.copy_(keep)
    assert pair.S == one.S == C * S
    lse_pair = cpu(E.lse_finalize(pair.m, pair.s, pair.e, C * S, lse_out=True)[1])
    lse_one = cpu(E.lse_finalize(one.m, one.s, one.e, C * S, lse_out=True)[1])
    Xh, Yh = cpu(Xt).astype(np.float64), cpu(Yt).astype(np.float64)
    lps, ses = [], []
    for s in range(S):
        for c in range(C):
            lp, se = _oracle_lp_se(_oracle_params(m, _unpack(eng, cpu(thetas[s, c]))), Xh, Yh)
            lps.append(lp)
            ses.append(se)
    # per point, against the float64 oracle: 2e-5 of max(1, |LSE|) (as the four-chain test);
    # the one-launch-per-sample fold meets the same bound
    ref_lse = _oracle_lse(np.stack(lps))
    tol = 2e-5 * np.maximum(1.0, np.abs(ref_lse))
    err_pair, err_one = np.abs(lse_pair - ref_lse), np.abs(lse_one - ref_lse)
    assert np.all(err_one < tol), float(np.max(err_one / tol))
    assert np.all(err_pair < tol), float(np.max(err_pair / tol))
    ll, rmse = pair.finalize(y_std=1.0)
    ref_ll, ref_rmse = O.predictive_summary(np.stack(lps), np.stack(ses))
    assert abs(ll - ref_ll) < 1e-4 and abs(rmse - ref_rmse) < 1e-5 * ref_rmse


@pytest.mark.parametrize("C,S", [(1, 5), (2, 4)])
def test_predictive_pairs_one_launch_equals_launch_per_pair(dev, C, S):
    """dgprf_forward_samples with the scratch of dgprf_forward_samples_scratch runs every sample pair
    in ONE launch (grid.z = pair), writes each sample's per-row log p / squared error to scratch
    and folds them in sample order with k_lse_fold_samples; without that scratch it launches the
    pair kernel once per pair and folds in place.  Both must give the same bits."""
    from dgprf import _native as N
    from dgprf import engine as E
    from dgprf.data import regression_data
    from dgprf.engine import ops
    n_test = 20_001  # the pair kernel applies from 16,384 rows (the lean tile kernel's range)
    Xt, Yt, _ = regression_data(n_test, CFG2["D"], seed=17, device=dev)
    m = _config2_model(21)
    eng = m._engine if C == 1 else _multi_chain_engine(m, C, seed=79)
    eng.build_omega()
    E.set_seed(22)
    thetas = torch.stack([E.normal((C, eng.layout.w_total), N.RNG_W) for _ in range(S)])
    Y2 = Yt if Yt.dim() == 2 else Yt[:, None]
    need = eng.forward_scratch(n_test, S)
    assert need is not None and need.numel() >= 2 * S * C * n_test
    outs = []
    for scr in (need, None):
        acc = [torch.full((C, n_test), -np.inf, device=dev), torch.zeros(C, n_test, device=dev),
               torch.zeros(C, n_test, device=dev)]
        ops().forward_samples(eng._plan_t(eng.layout), thetas, eng.omega, eng.der, Xt, None, Y2,
                              acc[0], acc[1], acc[2], scr)
        torch.cuda.synchronize()
        outs.append([cpu(a) for a in acc])
    for a, b in zip(outs[0], outs[1]):
        assert np.array_equal(a, b)
    assert np.isfinite(outs[0][0]).all() and (outs[0][1] > 0).all()


def _multi_chain_engine(m, C, seed):
    """C chains sharing model m's frequencies and hyper-parameters (one posterior)."""
    from dgprf import engine as E
    eng = m._engine
    me = E.Engine(eng.spec, C, seed=seed)
    me.z.copy_(eng.z)
    me.hyp.copy_(eng.hyp)
    me.lik_log_var_source = eng.lik_log_var_source
    me.build_omega()
    return me


def test_predictive_four_chains_and_eight_parts(dev):
    """An engine with C = 4 chains (k_forward_tiles with grid.y = 4) folds 2 samples per chain
    (finalize over parts = 4), and two such accumulator sets stacked as a two-rank gather
    (k_lse_finalize over parts = 8, S = 16): LL, RMSE and the per-point LSE against the oracle over
    all samples (utils_training.py:79-85 reduce_logsumexp over the stacked [S, N_t] matrix)."""
    from dgprf import _native as N
    from dgprf import engine as E
    from dgprf.data import regression_data
    from dgprf.predictive import PredictiveLSE
    n_test = 20_001
    Xt, Yt, _ = regression_data(n_test, CFG2["D"], seed=4, device=dev)
    m = _config2_model(5)
    me = _multi_chain_engine(m, 4, seed=77)
    accs, thetas = [], []
    E.set_seed(9)
    for part in range(2):
        acc = PredictiveLSE(me, Xt, Yt)
        for s in range(2):
            E.normal(None, N.RNG_W, out=me.theta)
            thetas.append(cpu(me.theta))
            acc.add_sample()
        accs.append(acc)
    Xh, Yh = cpu(Xt).astype(np.float64), cpu(Yt).astype(np.float64)
    lp_all, se_all = [], []
    for th in thetas:  # [4, w_total] per round
        for c in range(4):
            lp, se = _oracle_lp_se(_oracle_params(m, _unpack(me, th[c])), Xh, Yh)
            lp_all.append(lp)
            se_all.append(se)
    lp_all, se_all = np.stack(lp_all), np.stack(se_all)
    # one accumulator set: parts = 4 chains, 8 samples (rounds 0 and 1)
    ll4, rmse4 = accs[0].finalize(y_std=1.0)
    ref_ll4, ref_rmse4 = O.predictive_summary(lp_all[:8], se_all[:8])
    assert abs(ll4 - ref_ll4) < 1e-4 and abs(rmse4 - ref_rmse4) < 1e-5 * ref_rmse4
    # two sets stacked in rank order: parts = 8, S = 16
    cat = lambda k: torch.cat([getattr(a, k) for a in accs], dim=0)
    out, lse = E.lse_finalize(cat("m"), cat("s"), cat("e"), 16, y_std=2.0, lse_out=True)
    out = out.cpu().numpy()
    ref_ll8, ref_rmse8 = O.predictive_summary(lp_all, se_all, y_std=2.0)
    assert abs(out[0] - ref_ll8) < 1e-4 and abs(out[1] - ref_rmse8) < 1e-5 * ref_rmse8
    # per point: 2e-5 of the point's |LSE| (random N(0,1) weights put |log p| in the hundreds for
    # some points, where one fp32 ulp of log p is already ~3e-5); the 1e-4 bound is on the mean
    ref_lse = _oracle_lse(lp_all)  # lse_out is LSE_s log p (no y_std shift, include/dgprf.h)
    assert np.all(np.abs(cpu(lse) - ref_lse) < 2e-5 * np.maximum(1.0, np.abs(ref_lse)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_worker(rank, world, port, q, backend="gloo"):
    """One rank: 2 chains of its own (rank-keyed draws of W) over the shared test set and model,
    2 samples each; PredictiveLSE.finalize all-gathers the accumulators (gloo: host-staged, two
    ranks share the one GPU; nccl = RCCL: device tensors, one rank per GPU) and runs
    k_lse_finalize on the stacked [world * 2, n] rows.  The model comes from the helper bench.py
    uses (dgprf.distributed.chain_model): z and the hyper-parameters are gathered and must be
    bitwise equal on every rank (one posterior)."""
    from dgprf import _native as N
    from dgprf import engine as E
    from dgprf.data import regression_data
    from dgprf.distributed import chain_model, rank_seed
    from dgprf.predictive import PredictiveLSE
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    xfer = (lambda t: t) if backend == "nccl" else (lambda t: t.cpu())
    Xt, Yt, _ = regression_data(5_003, CFG2["D"], seed=6, device="cuda")
    m = chain_model(_build_config2, 8, rank)
    eng = m._engine
    eng.build_omega()
    for t in (eng.z, eng.hyp, eng.omega):  # one model on every rank
        parts = [torch.empty_like(xfer(t)) for _ in range(world)]
        dist.all_gather(parts, xfer(t))
        assert all(torch.equal(parts[0], p) for p in parts), "ranks built different models"
    seeds = [None] * world
    dist.all_gather_object(seeds, (eng.seed, float(eng.theta[0, 0])))
    assert len(set(seeds)) == world, "every rank's chain needs its own noise key and W init"
    me = _multi_chain_engine(m, 2, seed=rank_seed(1, rank))
    E.set_seed(rank_seed(2, rank))
    acc = PredictiveLSE(me, Xt, Yt)
    th = []
    for s in range(2):
        E.normal(None, N.RNG_W, out=me.theta)
        th.append(cpu(me.theta))
        acc.add_sample()
    ll, rmse = acc.finalize(y_std=1.3)
    q.put((rank, np.stack(th), ll, rmse))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,backend", [(2, "gloo"), (1, "nccl")])
def test_predictive_two_ranks_gather_and_finalize(dev, world, backend):
    """PredictiveLSE.finalize (gather_accumulators + k_lse_finalize) on the GPU: world_size 2 over
    gloo (both ranks on the one GPU), and a one-rank nccl (= RCCL) group, whose all-gather runs the
    device-tensor branch the 8-GPU runs take (dgprf/distributed.py); every rank reports the same
    LL / RMSE, equal to the oracle over all world x 2 x 2 samples."""
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = mp.spawn(_rank_worker, args=(world, port, q, backend), nprocs=world, join=False)
    # drain the queue before joining: a child cannot exit while its queued arrays sit in the pipe
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda r: r[0])
    procs.join()
    m = _config2_model(8)
    from dgprf.data import regression_data
    Xt, Yt, _ = regression_data(5_003, CFG2["D"], seed=6, device=dev)
    Xh, Yh = cpu(Xt).astype(np.float64), cpu(Yt).astype(np.float64)
    eng = m._engine
    lp_all, se_all = [], []
    for _, th, _, _ in res:                       # rank order, then sample, then chain
        for s in range(th.shape[0]):
            for c in range(th.shape[1]):
                lp, se = _oracle_lp_se(_oracle_params(m, _unpack(eng, th[s, c])), Xh, Yh)
                lp_all.append(lp)
                se_all.append(se)
    ref_ll, ref_rmse = O.predictive_summary(np.stack(lp_all), np.stack(se_all), y_std=1.3)
    for _, _, ll, rmse in res:
        assert abs(ll - ref_ll) < 1e-4 and abs(rmse - ref_rmse) < 1e-5 * ref_rmse
    assert all(r[2] == res[0][2] and r[3] == res[0][3] for r in res)
