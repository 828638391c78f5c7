"""The N>1 predictive exchange on CPU: world_size-2 gloo ranks each fold their own chains'
samples into LSE accumulators, gather_accumulators (the RCCL all-gather on the GPU box) stacks
them in rank order, and the combined log-sum-exp equals the oracle over all samples."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dgprf import distributed as D
from oracle import dgp_oracle as O


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _lse_acc(lp):
    """Online (max, sum) over samples exactly as k_forward_rows folds them."""
    m = np.full(lp.shape[1], -np.inf, dtype=np.float64)
    s = np.zeros(lp.shape[1])
    for row in lp:
        m1 = np.maximum(m, row)
        s = s * np.exp(m - m1) + np.exp(row - m1)
        m = m1
    return m, s


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(100 + rank)
    C, n, S = 2, 37, 5                    # 2 chains per rank, 5 samples each
    lp = rng.normal(-1.0, 0.7, size=(C, S, n))
    se = rng.random((C, S, n))
    ms, ss = zip(*[_lse_acc(lp[c]) for c in range(C)])
    m = torch.tensor(np.stack(ms))
    s = torch.tensor(np.stack(ss))
    e = torch.tensor(se.sum(axis=1))
    calls = []  # every collective gather_accumulators issues
    for name in ("all_gather", "all_reduce", "all_gather_into_tensor", "broadcast"):
        f = getattr(dist, name)
        setattr(dist, name, (lambda f, name: lambda *a, **k: (calls.append(name), f(*a, **k))[1])(
            f, name))
    M, Sa, E, S_tot = D.gather_accumulators(m, s, e, C * S)
    assert calls == ["all_gather"], calls  # (m | s | e | S) packed into one exchange
    M2, S2, E2, _ = D.gather_accumulators(m, s, None, C * S)  # a softmax model: no se sums
    assert E2 is None and torch.equal(M2, M) and torch.equal(S2, Sa)
    assert M.shape == (world * C, n) and S_tot == world * C * S
    if rank == 0:
        q.put((M.numpy(), Sa.numpy(), E.numpy(), S_tot))
    assert D.world()[:2] == (rank, world)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_predictive_gather():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.spawn(_worker, args=(world, port, q), nprocs=world, join=True)
    M, Sa, E, S_tot = q.get()
    # every rank's raw samples, regenerated exactly as the workers drew them
    all_lp, all_se = [], []
    for r in range(world):
        rng = np.random.default_rng(100 + r)
        lp = rng.normal(-1.0, 0.7, size=(2, 5, 37))
        se = rng.random((2, 5, 37))
        all_lp.append(lp.reshape(-1, 37))
        all_se.append(se.reshape(-1, 37))
    lp, se = np.concatenate(all_lp), np.concatenate(all_se)
    ll_ref, rmse_ref = O.predictive_summary(lp, se, y_std=1.0)
    mx = M.max(axis=0)
    lse = mx + np.log((Sa * np.exp(M - mx)).sum(axis=0))
    ll = np.mean(lse - np.log(S_tot))
    rmse = np.sqrt(E.sum() / (S_tot * 37))
    assert np.isclose(ll, ll_ref) and np.isclose(rmse, rmse_ref)


def test_rank_seeds_distinct():
    seeds = {D.rank_seed(1234, r) for r in range(64)}
    assert len(seeds) == 64 and all(0 <= s < 2 ** 64 for s in seeds)
