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
    collective (the code path of the N-GPU runs).

    ONE collective: every rank packs (m | s | e | S) into one contiguous buffer and all-gathers it
    (a latency-bound exchange over xGMI — one RCCL call instead of three all-gathers and an
    all-reduce); S, a sample count < 2^24, is exact in the accumulators' float type."""
    if not (dist.is_available() and dist.is_initialized()):
        return m, s, e, S_local
    W = dist.get_world_size(group)
    if not 0 <= int(S_local) < (1 << 24):
        raise ValueError(f"sample count {S_local} outside the packed range")
    # RCCL ("nccl") gathers device tensors over xGMI; gloo (CPU tests, or several ranks sharing one
    # GPU in the GPU tests) gathers host tensors, so its device accumulators are staged through host
    host = dist.get_backend(group) == "gloo"
    acc = [m, s] + ([e] if e is not None else [])
    C, n = m.shape
    k = len(acc)
    buf = torch.empty(k * C * n + 1, dtype=m.dtype, device=m.device)
    for i, t in enumerate(acc):
        buf[i * C * n:(i + 1) * C * n].copy_(t.reshape(-1))
    buf[-1] = float(S_local)
    src = buf.cpu() if host else buf
    parts = torch.empty(W, src.numel(), dtype=src.dtype, device=src.device)
    dist.all_gather(list(parts.unbind(0)), src, group=group)
    parts = parts.to(m.device)
    out = [parts[:, i * C * n:(i + 1) * C * n].reshape(W * C, n) for i in range(k)]
    S = float(parts[:, -1].double().sum().item())
    return out[0], out[1], (out[2] if e is not None else None), S
