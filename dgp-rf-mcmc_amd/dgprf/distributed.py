"""Chain-parallel multi-GPU plumbing: one process per GPU, torch.distributed (RCCL) only at
prediction time.  Chains are independent, so the sampling phase has no
collective; the predictive accumulators are all-gathered once."""
import os

import torch
import torch.distributed as dist

_M64 = (1 << 64) - 1


def world():
    """(rank, world_size, local_rank) from torch.distributed or the launcher env."""
    if dist.is_available() and dist.is_initialized():
        r, w = dist.get_rank(), dist.get_world_size()
    else:
        r, w = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    return r, w, int(os.environ.get("LOCAL_RANK", r))


def rank_seed(seed, rank):
    """Independent Philox key per rank (splitmix64 of seed and rank)."""
    z = (int(seed) + 0x9E3779B97F4A7C15 * (int(rank) + 1)) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def chain_model(build, model_seed, rank):
    """This rank's chain of ONE posterior.

    The model — RF frequencies z, kernel / likelihood hyper-parameters, everything `build()` draws
    at construction (layers/rf_layers.py:21-22) — comes from the rank-independent `model_seed`, so
    every rank samples the same fixed-z model, as the reference scores successive samples of one
    model (experiments/utils_training.py:62-65,79-85).  Only the chain's own state folds the rank:
    the Philox key of its step noise, its W initialisation (layers/GP_weight_layers.py:9) and the
    momenta drawn later by precond_update (models/dgp.py:235-240)."""
    from . import _native as N
    from . import engine as E
    E.set_seed(model_seed)
    m = build()
    eng = m._engine
    E.set_seed(rank_seed(model_seed, rank))
    eng.seed = E.engine_key()
    E.normal(None, N.RNG_W, out=eng.theta)
    return m


def gather_accumulators(m, s, e, S_local, group=None):
    """All-gather per-rank LSE accumulators [C, n] -> [W*C, n] in rank order, and sum S.  Without
    a process group the local accumulators are the whole; a one-rank group still runs the
    collective (the code path of the N-GPU runs)."""
    if not (dist.is_available() and dist.is_initialized()):
        return m, s, e, S_local
    W = dist.get_world_size(group)
    # RCCL ("nccl") gathers device tensors over xGMI; gloo (CPU tests, or several ranks sharing one
    # GPU in the GPU tests) gathers host tensors, so its device accumulators are staged through host
    host = dist.get_backend(group) == "gloo"

    def ag(t):
        src = t.contiguous().cpu() if host else t.contiguous()
        parts = [torch.empty_like(src) for _ in range(W)]
        dist.all_gather(parts, src, group=group)
        return torch.cat(parts, dim=0).to(t.device)

    S = torch.tensor([float(S_local)], dtype=torch.float64, device="cpu" if host else m.device)
    dist.all_reduce(S, group=group)
    return ag(m), ag(s), (ag(e) if e is not None else None), float(S.item())
