#!/usr/bin/env python
"""bench.py — SGHMC steps/s + predictive samples/s of the L=3, RF=1024 DGP (BASELINE config 2).

A "step" is one DGP_RF.sgmcmc_update (models/dgp.py:184-216): on-device minibatch of B=200 rows
from the device-resident N=1e6 x 8 dataset, forward through 3 RBF-RF layers, Gaussian
likelihood, analytic backward, SGHMC update with Philox noise — one chain per GPU (weak scaling,
chain-parallel).  A "predictive sample" is the full forward of the N_t=1e5 test set for one
posterior sample + log p + se + the online log-sum-exp accumulation (utils_training.py:79-85).

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N --steps K --warmup W
Rank 0 prints ONE JSON line.  `--gpus N` is authoritative: without a launcher (WORLD_SIZE unset)
and N > 1 the process starts the N ranks itself (torch.distributed.run as a child, before any GPU
call) and exits with its status; under a launcher WORLD_SIZE must equal N.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "dgp-rf-mcmc_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "SGHMC steps/sec + predictive samples/sec, L=3 RF=1024 DGP, 1/2/4/8 GPU"
FP32_MFMA_PEAK = 157.3e12   # MI355X_MICROARCH.md: v_mfma_f32_16x16x4_f32 dense peak (FLOP/s)
HBM_PEAK = 8.0e12           # MI355X_MICROARCH.md: HBM3E spec (B/s)
# MI355X_MICROARCH.md per-instruction table: v_sin_f32 / v_cos_f32 issue 8 cycles per 64-lane wave
# instruction on a SIMD; 256 CUs x 4 SIMDs at the 2.4 GHz peak clock
TRANS_PER_S = 1024 * 64 / 8 * 2.4e9
PROFILES = os.path.join(ROOT, "profiles", "r06")   # this round's committed rocprofv3 evidence

CFG = dict(L=3, n_rf=1024, n_gp=[8, 8, 1], D=8, N=1_000_000, B=200, N_test=100_000,
           variance=0.1, lr=0.01, beta=0.9, T=1.0)


def step_flops(B, d, R, P, g):
    """per-kernel algorithmic FLOPs of one step (per layer)."""
    fwd = [2 * B * (d[l] * R[l] + P[l] * g[l]) for l in range(len(d))]
    bwd = [2 * B * P[l] * g[l] + (2 * B * (P[l] * g[l] + R[l] * d[l]) if l > 0 else 0)
           for l in range(len(d))]
    return fwd, bwd


def pred_flops(n, d, R, P, g):
    return n * sum(2 * (d[l] * R[l] + P[l] * g[l]) for l in range(len(d)))


def cpu_model():
    """`model name` of the host CPU (/proc/cpuinfo, as lscpu reports it)."""
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_threads():
    """BLAS threads numpy actually runs with (threadpoolctl), and the reason for that count."""
    try:
        from threadpoolctl import threadpool_info
        n = max([int(i.get("num_threads", 1)) for i in threadpool_info()
                 if i.get("user_api") == "blas"] or [1])
    except Exception:
        n = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    return n


def cpu_baseline(runs=5, warm=50, timed=1000, pred_samples=5):
    """The reference algorithm, op for op, on the host (oracle/dgp_oracle.py in float32 numpy):
    TensorFlow is not installed here or on the GPU box, so this restatement is the CPU proxy.
    BASELINE.md §3 protocol: `warm` warm-up steps then `timed` timed steps, median of `runs` runs;
    predictive: `pred_samples` full N_test = 1e5-row samples (in 10k-row chunks)."""
    from oracle import dgp_oracle as O
    rng = np.random.default_rng(0)
    f32 = np.float32
    R, g = CFG["n_rf"], CFG["n_gp"]
    p = O.Params(8, 1, [R] * 3, g, ["RBF"] * 3, "gaussian", False, rng=rng,
                 lik_log_var=np.log(CFG["variance"]), dtype=np.float32)
    n_data = 200_000   # host copy of the synthetic regression data (same distribution)
    X = rng.standard_normal((n_data, 8)).astype(f32)
    a = rng.standard_normal((8, 1)).astype(f32) / f32(np.sqrt(8))
    Y = (np.sin(X @ a) + f32(0.1) * rng.standard_normal((n_data, 1)).astype(f32)).astype(f32)
    Y = ((Y - Y.mean()) / Y.std()).astype(f32)
    m = [rng.standard_normal(w.shape).astype(f32) for w in p.W]
    N, B = CFG["N"], CFG["B"]

    def steps(k):
        nonlocal m
        for _ in range(k):
            idx = rng.integers(0, n_data, B)
            xi = [rng.standard_normal(w.shape).astype(f32) for w in p.W]
            m = O.sgmcmc_step(p, m, X[idx], Y[idx], f32(N), f32(CFG["lr"]), f32(CFG["beta"]),
                              f32(CFG["T"]), [f32(1.0)] * 3, xi)

    rates = []
    for _ in range(runs):
        steps(warm)
        t0 = time.perf_counter()
        steps(timed)
        rates.append(timed / (time.perf_counter() - t0))
    step_rate = float(np.median(rates))
    Xt = rng.standard_normal((CFG["N_test"], 8)).astype(f32)
    Yt = rng.standard_normal((CFG["N_test"], 1)).astype(f32)
    t0 = time.perf_counter()
    for _ in range(pred_samples):
        for i in range(0, CFG["N_test"], 10_000):
            O.eval_log_likelihood_and_se(p, Xt[i:i + 10_000], Yt[i:i + 10_000])
    pred_rate = pred_samples / (time.perf_counter() - t0)
    return {"value": round(step_rate, 2), "unit": "steps/s", "cores": cpu_threads(), "kind": "port",
            "cpu_model": cpu_model(), "host_cpus": os.cpu_count(),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "threads_note": "BLAS threads numpy runs with (threadpoolctl); on the GPU box the job's "
                            "CPU share is 16 (OMP_NUM_THREADS=16 set by the harness) while "
                            "os.cpu_count() reports the whole host",
            "protocol": f"{warm} warm-up + {timed} timed steps, median of {runs} runs "
                        f"({', '.join(f'{r:.1f}' for r in rates)} steps/s); predictive "
                        f"{pred_samples} full samples",
            "sample": "SGHMC steps of config 2 (B=200, L=3, n_rf=1024, float32 numpy op-for-op "
                      "restatement of models/dgp.py:184-216, injected N(0,1) noise); predictive: "
                      "forward + log p + se of all 1e5 test rows per sample",
            "predictive_samples_per_s": round(pred_rate, 4),
            "note": "BLAS matmuls use the listed threads; numpy elementwise/trig is single-threaded"}


def _short(name):
    """Kernel name without 'void ', namespaces and the argument list (rocprofv3 CSV names)."""
    import re
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    name = re.sub(r"\([^()]*\)$", "", name)  # the parameter list
    return re.sub(r"\w+::", "", name)


def pmc_traffic(prefix):
    """HBM-side bytes per launch of the kernels named `prefix...` (dispatch-weighted mean), from the
    committed rocprofv3 FETCH_SIZE / WRITE_SIZE passes (profiles/r05/pmc_traffic.json, made by
    scripts/gpu_profile_round.sh; FETCH doubled per MI355X_MICROARCH.md §HBM).  None if absent."""
    path = os.path.join(PROFILES, "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    with open(path) as fh:
        ks = json.load(fh)["kernels"]
    sel = [v for k, v in ks.items() if (_short(k) + "<").startswith(prefix + "<") and "dispatches" in v]
    n = sum(v["dispatches"] for v in sel)
    return round(sum(v["traffic"] * v["dispatches"] for v in sel) / n) if n else None


def rocprof_avg_us(prefix, fname="kernel_stats_bench.csv"):
    """Dispatch-weighted average duration (us) of the kernels named `prefix<...>` in the committed
    rocprofv3 --kernel-trace --stats summary of this bench (profiles/r05/kernel_stats_bench.csv);
    None if absent.  Traced durations include each dispatch's own launch overhead."""
    import csv
    path = os.path.join(PROFILES, fname)
    if not os.path.exists(path):
        return None
    n = tot = 0.0
    with open(path) as fh:
        for r in csv.DictReader(fh):
            name = _short(r["Name"])
            if name == prefix or name.startswith(prefix + "<"):
                n += float(r["Calls"])
                tot += float(r["TotalDurationNs"])
    return round(tot / n / 1e3, 3) if n else None


def bench_config(cfg, dev, rank, world, barrier_sync, max_over_ranks, steps):
    """Steps/s and predictive samples/s of BASELINE config 3, 4 or 5 (dgprf.data.CONFIGS): the full
    model shape on synthetic data of the config's size, one chain per GPU, graph-replayed steps."""
    from dgprf.data import CONFIGS, classification_data, regression_data
    from dgprf.distributed import chain_model, rank_seed
    from dgprf.predictive import PredictiveLSE
    from likelihoods import Gaussian, Softmax
    from models.dgp import DGP_RF
    c = CONFIGS[cfg]
    n, nt = c["n"], c["n_test"]
    if c["likelihood"] == "softmax":
        X, Y = classification_data(n, c["d_in"], c["d_out"], seed=0, device=dev)
        Xt, Yt = classification_data(nt, c["d_in"], c["d_out"], seed=1, device=dev)
        lik = Softmax()
    else:
        X, Y, a = regression_data(n, c["d_in"], seed=0, device=dev)
        Xt, Yt, _ = regression_data(nt, c["d_in"], seed=1, device=dev, a=a)
        lik = Gaussian(variance=c["variance"])
    # one model (z, hyper-parameters) on every rank; the rank folds only into its chain's state
    m = chain_model(lambda: DGP_RF(c["d_in"], c["d_out"], n_hidden_layers=len(c["kinds"]),
                                   n_rf=c["n_rf"], n_gp=c["n_gp"], likelihood=lik,
                                   kernel_type_list=c["kinds"]), 20 + cfg, rank)
    m.precond_update(None, n, precond_type="identity")
    run = dict(batch_size=c["batch"], lr=c["lr"], momentum_decay=c["beta"], temperature=c["T"],
               steps_per_graph=100, perm_seed=rank_seed(cfg, rank))
    m.run_sgmcmc(X, Y, n, 100, **run)
    pl = m._engine.layout
    eng = m._engine
    L = len(c["kinds"])
    d, R, P, g = list(pl.d[:L]), list(pl.n_rf[:L]), list(pl.P[:L]), list(pl.n_gp[:L])
    fwd_f, bwd_f = step_flops(c["batch"], d, R, P, g)
    # a wide first layer's resident X Omega_1 (W-only steps gather its rows; SURVEY §8d counts the
    # step's A_1 = X_B Omega_1 GEMM): the projection of the whole training set is recomputed INSIDE
    # the timed region (into the buffer the captured graphs hold), so the step rate carries its
    # one-off cost amortised over the timed steps; its time alone is measured beside it
    resident = pl.a0_off >= 0 and eng.dataset_a1(X) is not None
    proj_ms = None
    if resident:
        eng.invalidate_a1()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        eng.dataset_a1(X)
        e1.record()
        torch.cuda.synchronize()
        proj_ms = e0.elapsed_time(e1)
        eng.invalidate_a1()  # the timed run_sgmcmc recomputes it
    barrier_sync()
    t0 = time.perf_counter()
    m.run_sgmcmc(X, Y, n, steps, **run)
    barrier_sync()
    t_s = max_over_ranks(time.perf_counter() - t0)
    assert torch.isfinite(m._engine.theta).all(), f"config {cfg} chain diverged"
    a1 = None
    a1_skip = 0  # per step: the A_1 GEMM FLOPs the step does not execute
    proj_fl = 0  # per timed region: the projection FLOPs it executes instead
    if pl.a0_off >= 0:  # wide first layer
        a1_fl = 2 * c["batch"] * d[0] * R[0]
        a1_skip = a1_fl if resident else 0
        proj_fl = 2 * n * d[0] * R[0] if resident else 0
        # the per-step A_1 GEMM the resident projection replaces (hipEvents, dgprf_profile_step)
        prof = eng.profile_step(X, Y, c["batch"], n, c["lr"], c["beta"], c["T"], reps=100)
        g_us = max(prof["agemm"] - prof["empty"], 0.0) * 1e3
        excl_us = (t_s - (proj_ms or 0.0) * 1e-3) * 1e6 / steps
        a1 = {"form": ("resident: X Omega_1 of the whole dataset kept in HBM (Engine.dataset_a1, "
                       f"{n} x {R[0]} fp32), each step gathers its minibatch's rows; the "
                       "projection is recomputed inside the timed region (us_per_step includes "
                       "it, amortised over the timed steps)" if resident else
                       "per-step A_1 GEMM (k_agemm, two K parts)"),
              "dataset_projection_ms": round(proj_ms, 3) if proj_ms is not None else None,
              "dataset_projection_gflop": round(2 * n * d[0] * R[0] / 1e9, 2),
              "us_per_step_excl_projection": round(excl_us, 2) if resident else None,
              "step_gemm_us_replaced": round(g_us, 2), "step_gemm_mflop": round(a1_fl / 1e6, 1),
              "step_mfma_frac_excl_a1": round((sum(fwd_f) + sum(bwd_f) - a1_fl) /
                                              ((excl_us if resident else t_s * 1e6 / steps - g_us)
                                               * 1e-6) / FP32_MFMA_PEAK, 4)}
    # configs 3 / 5 name 8 chains (on 8 GPUs in the reference): here 8 chains per GPU in one launch
    # sequence of the multi-chain engine (its own slice widths), started from this
    # chain's state; aggregate chain-steps/s, reported beside the one-chain rate.  Configs 4 / 5
    # also at 64 chains per GPU (the throughput regime: one backward row group per chain)
    def chains_leg(C, reps):
        from dgprf import engine as E
        eng = m._engine
        me = E.Engine(eng.spec, C, seed=rank_seed(40 + cfg + C, rank))
        me.z.copy_(eng.z)
        me.hyp.copy_(eng.hyp)
        me.theta.copy_(eng.theta.expand(C, -1))
        me.init_moments()
        me.lik_log_var_source = eng.lik_log_var_source
        me.build_omega()
        gph = me.graph(X, Y, c["batch"], n, c["lr"], c["beta"], c["T"], 50)
        gph.launch()
        mpl = me.plan_ws(c["batch"])[0]
        # the chains share Omega_1, so they share one resident projection: built with the graph,
        # counted below as one recompute per timed region (its time from the one-chain leg)
        res = resident and mpl.a0_off >= 0 and me.dataset_a1(X) is not None
        barrier_sync()
        t0 = time.perf_counter()
        for _ in range(reps):
            gph.launch()
        barrier_sync()
        tc = max_over_ranks(time.perf_counter() - t0)
        assert torch.isfinite(me.theta).all(), f"config {cfg} {C}-chain run diverged"
        cs = C * reps * 50
        t_inc = tc + ((proj_ms or 0.0) * 1e-3 if res else 0.0)
        ex = cs * (sum(fwd_f) + sum(bwd_f) - (a1_skip if res else 0)) + (proj_fl if res else 0)
        out = {"chains_per_gpu": C, "slices_per_layer": list(mpl.ns[:L]),
               "bwd_row_groups_per_chain": int(mpl.n_gw_rows),
               "chain_steps_per_s": round(world * cs / tc, 1),
               "us_per_step_all_chains": round(tc * 1e6 / (reps * 50), 2),
               "chain_steps_per_s_incl_projection": round(world * cs / t_inc, 1) if res else None,
               "step_mfma_frac": round(ex / t_inc / FP32_MFMA_PEAK, 4)}
        del gph, me
        torch.cuda.empty_cache()
        return out
    chains8 = chains_leg(8, 4) if cfg in (3, 5) else None
    chains64 = chains_leg(64, 3) if cfg in (4, 5) else None
    # S posterior samples (the chain's W at S successive steps) scored by ONE add_samples call:
    # every sample in one launch of the predictive kernel (grid.z = sample), then the fold; S = the
    # reference driver's default sample count (60), config 5 (1e6 test rows, ~27 ms per sample) 3
    S = 3 if cfg == 5 else 60
    th_all = [m._engine.theta.clone()]
    for _ in range(S - 1):
        m.run_sgmcmc(X, Y, n, 1, **run)
        th_all.append(m._engine.theta.clone())
    th_all = torch.stack(th_all)
    acc = PredictiveLSE(m._engine, Xt, Yt)
    acc.add_samples(th_all)  # scratch and first launch outside the clock
    # a wide first layer: the test set's X Omega_1 (shared by every sample, Omega_1 being fixed,
    # layers/rf_layers.py:21-22) is recomputed inside the clock, as the reference's driver scores
    # each sample from scratch (experiments/utils_training.py:63)
    pred_a1_shared = pl.a0_off >= 0 and m._engine.dataset_a1(Xt) is not None
    ev2, ev3 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    acc = PredictiveLSE(m._engine, Xt, Yt)
    torch.cuda.synchronize()
    ev2.record()
    acc.add_samples(th_all, build=False)  # projection cached: the samples alone
    ev3.record()
    torch.cuda.synchronize()
    k_ms_excl = ev2.elapsed_time(ev3) / S
    acc = PredictiveLSE(m._engine, Xt, Yt)
    if pred_a1_shared:
        m._engine.invalidate_a1()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier_sync()
    t0 = time.perf_counter()
    ev0.record()
    acc.add_samples(th_all, build=False)
    ev1.record()
    # the config's predictive ends with the accumulator all-gather over the ranks (RCCL over xGMI
    # under nccl) and the device log-sum-exp combine (utils_training.py:79-85): inside the region
    barrier_sync()
    t1 = time.perf_counter()
    ll, _ = acc.finalize(y_std=1.0)
    barrier_sync()
    t_fin = max_over_ranks(time.perf_counter() - t1)
    t_p = max_over_ranks(time.perf_counter() - t0)
    k_ms = ev0.elapsed_time(ev1) / S
    fp = pred_flops(nt, d, R, P, g)  # SURVEY §8d per sample (layer 0's X_test Omega_1 included)
    a1_pred = 2 * nt * d[0] * R[0] if pred_a1_shared else 0
    # executed in the region: every sample's layers without the shared projection, plus it once
    fp_exec = S * (fp - a1_pred) + a1_pred
    out = {"workload": f"{L}-layer {'/'.join(c['kinds'])} n_rf={c['n_rf'][0]} g={c['n_gp']} "
                       f"D={c['d_in']} N={n} B={c['batch']} {c['likelihood']}",
           "steps_per_s": round(world * steps / t_s, 1),
           "us_per_step": round(t_s * 1e6 / steps, 2),
           "step_mflop": round((sum(fwd_f) + sum(bwd_f)) / 1e6, 2),
           # executed FLOPs: without the A_1 GEMM when the step gathers resident rows instead
           "step_mfma_frac": round((steps * (sum(fwd_f) + sum(bwd_f) - a1_skip) + proj_fl) / t_s /
                                   FP32_MFMA_PEAK, 4),
           "predictive_samples_per_s": round(world * S / t_p, 3), "n_test": nt,
           "predictive_finalize_ms": round(t_fin * 1e3, 3),
           "predictive_finalize": f"all-gather of the [chains, {nt}] (max, sum, se) accumulators "
                                  f"over {world} rank(s) + device LSE combine, inside the timed "
                                  "predictive region",
           "test_loglik": round(ll, 5),
           "predictive_kernel_ms": round(k_ms, 3),
           "predictive_mfma_frac": round(fp_exec / (S * k_ms * 1e-3) / FP32_MFMA_PEAK, 4),
           "predictive_flops_per_sample": int(fp_exec // S),
           "predictive_flops_note": ("executed FLOPs per sample: the samples' layers plus the "
                                     "test set's X Omega_1 once per call (computed inside the "
                                     "timed region), amortised over the call's samples; SURVEY "
                                     "§8d counts that projection per sample "
                                     f"({int(fp)} FLOP/sample), work a fixed Omega_1 makes "
                                     "redundant" if pred_a1_shared else
                                     "SURVEY §8d FLOPs per sample"),
           "predictive_a1": ({"form": "X_test Omega_1 resident, shared by every sample; "
                                      "recomputed inside the timed region",
                              "samples_per_call": S,
                              "predictive_kernel_ms_excl_projection": round(k_ms_excl, 3),
                              "s8d_flops_per_sample": int(fp)} if pred_a1_shared else None),
           "a1_gemm": a1,
           "chains8_per_gpu": chains8, "chains64_per_gpu": chains64}
    del m, acc, X, Y, Xt, Yt
    torch.cuda.empty_cache()
    return out


def eager_api(model, X, Y, N_, B, calls=2000, n_batches=50):
    """The drop-in per-call path the reference's driver runs (experiments/utils_training.py:45-61):
    one model.sgmcmc_update(x, y, N, ...) call per minibatch (models/dgp.py:184-216), each a
    Python -> torch-op -> C-ABI call launching the step's kernels; minibatches device-resident
    (slices of the HBM dataset) and host numpy arrays copied per call, as a tf.data loader hands
    them over.  Also precond_update(ds, N, K_batches=32) (run every epoch by the reference,
    experiments/utils_training.py:42).  The model's momenta and masses are restored afterwards."""
    eng = model._engine
    keep = (eng.theta.clone(), eng.mom.clone(), eng.mass.clone(), int(eng.step_ctr))
    dev_b = [(X[i * B:(i + 1) * B], Y[i * B:(i + 1) * B]) for i in range(n_batches)]
    host_b = [(x.cpu().numpy(), y.cpu().numpy()) for x, y in dev_b]
    kw = dict(lr=CFG["lr"], momentum_decay=CFG["beta"], temperature=CFG["T"])
    out = {}
    for name, batches in (("device_batches", dev_b), ("host_numpy_batches", host_b)):
        for i in range(50):
            model.sgmcmc_update(*batches[i % n_batches], N_, **kw)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(calls):
            model.sgmcmc_update(*batches[i % n_batches], N_, **kw)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        out[name] = {"steps_per_s": round(calls / dt, 1), "us_per_call": round(dt * 1e6 / calls, 2),
                     "calls": calls}
    ds = [dev_b[i % n_batches] for i in range(32)]
    model.precond_update(ds, N_, K_batches=32)  # warm (workspace / scratch allocation)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    model.precond_update(ds, N_, K_batches=32)
    torch.cuda.synchronize()
    out["precond_update_k32_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
    eng.theta.copy_(keep[0])
    eng.mom.copy_(keep[1])
    eng.mass.copy_(keep[2])
    eng.step_ctr.fill_(keep[3])
    out["method"] = ("model.sgmcmc_update per call, B=200 config-2 minibatches (50 distinct, "
                     "cycled), wall time over `calls` calls closed by a synchronize; Omega built "
                     "only when stale; precond_update: 32 gradient minibatches + Welford + masses")
    return out


def driver_loop(dev, rank, X, Y, Xt, Yt, epochs=6, start=2, per_cycle=2):
    """The reference's driver end to end (experiments/utils_training.py:11-88 regression_train) on
    config 2's data: every epoch precond_update(rmsprop, K_batches=32) (:42) then one epoch of
    SGHMC steps (N / B = 5,000 minibatches, burn-in at T = 0 then the cosine cycle, :45-61 — one
    hipGraph replay per epoch here), and at each cycle end the whole 1e5-row test set scored
    (eval_log_likelihood_and_se, :62-67); the [S, N_test] log p / squared errors it returns
    summarised at the end (:79-85).  `epochs` / `start` / `per_cycle` shrink the reference's
    5000 / 2000 / 50 to a bench-sized run.  Timed twice from the same step counter and permutation
    seed (so the second call replays the graphs the first captured); the split comes from a third
    run with each phase bracketed by synchronisations."""
    import contextlib
    import io
    from dgprf.distributed import chain_model
    from experiments.utils_training import regression_train
    from likelihoods import Gaussian
    from models.regression_model import RegressionDGP
    model = chain_model(lambda: RegressionDGP(CFG["D"], 1, n_hidden_layers=CFG["L"],
                                              n_rf=CFG["n_rf"], n_gp=CFG["n_gp"],
                                              likelihood=Gaussian(variance=CFG["variance"])),
                        2, rank)
    kw = dict(data=(X, Y, Xt, Yt), batch_size=CFG["B"], lr_0=CFG["lr"],
              momentum_decay=CFG["beta"], full_bayesian=False, precond_type="rmsprop",
              K_batches=32, second_moment_centered=False, total_epochs=epochs,
              start_sampling_epoch=start, epochs_per_cycle=per_cycle, print_epoch_cycle=10 ** 9)
    eng = model._engine
    split = {"precond": 0.0, "steps": 0.0, "eval": 0.0}

    def run(timed_split=False):
        eng.step_ctr.zero_()  # the same schedule clock (start_step) -> the cached graphs
        np.random.seed(1234)  # the same DeviceDataset permutation seed (perm_seed)
        if timed_split:
            for name, attr in (("precond", "precond_update"), ("steps", "run_sgmcmc"),
                               ("eval", "eval_log_likelihood_and_se")):
                f = getattr(model, attr)

                def w(*a, _f=f, _n=name, **k):
                    torch.cuda.synchronize()
                    t = time.perf_counter()
                    r = _f(*a, **k)
                    torch.cuda.synchronize()
                    split[_n] += time.perf_counter() - t
                    return r
                setattr(model, attr, w)
        torch.cuda.synchronize()
        t = time.perf_counter()
        with contextlib.redirect_stdout(io.StringIO()):
            log_p, mse = regression_train(model, **kw)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        if timed_split:
            for attr in ("precond_update", "run_sgmcmc", "eval_log_likelihood_and_se"):
                delattr(model, attr)
        return dt, log_p, mse

    first, _, _ = run()
    dt, log_p, mse = run()
    run(timed_split=True)
    assert torch.isfinite(eng.theta).all(), "driver chain diverged"
    ipe = X.shape[0] // CFG["B"]
    S = log_p.shape[0]
    ll = float((torch.logsumexp(log_p, 0) - math.log(S)).mean())
    return {"function": "experiments.utils_training.regression_train",
            "epochs": epochs, "start_sampling_epoch": start, "epochs_per_cycle": per_cycle,
            "steps_per_epoch": ipe, "samples_scored": S, "n_test": int(Xt.shape[0]),
            "precond": "rmsprop, K_batches=32, every epoch",
            "epochs_per_s": round(epochs / dt, 3), "s_per_call": round(dt, 4),
            "effective_steps_per_s": round(epochs * ipe / dt, 1),
            "first_call_s": round(first, 4),
            "first_call_note": "the first call also captures and instantiates the epoch graphs "
                               f"({ipe} steps each); later calls with the same schedule replay them",
            "per_epoch_ms": {k: round(v * 1e3 / epochs, 3) for k, v in split.items()},
            "per_sample_eval_ms": round(split["eval"] * 1e3 / max(S, 1), 3),
            "split_method": "third call with each phase bracketed by torch.cuda.synchronize()",
            "test_loglik": round(ll, 5), "test_rmse": round(float(torch.sqrt(mse.mean())), 5)}


def launch_boundary_us(dev, n=400):
    """Cost of one dependent kernel boundary inside a graph, measured live: a torch CUDA graph of
    n back-to-back one-element kernels on one stream, replayed; device time per kernel."""
    t = torch.zeros(1, device=dev)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        for _ in range(3):
            t.add_(1.0)
    torch.cuda.current_stream(dev).wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            t.add_(1.0)
    g.replay()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = None
    for _ in range(5):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize(dev)
        v = e0.elapsed_time(e1) * 1e3 / n
        best = v if best is None else min(best, v)
    del g
    return best


def b_sweep(model, X, Y, N_, batches, d, R, P, g):
    """SURVEY §8d B-sweep on the benchmark model: graph-replayed SGHMC steps at each minibatch size
    (steps/s and the step's fraction of the fp32 MFMA peak from the algorithmic FLOPs)."""
    out = {}
    for B, k in batches:
        run = dict(batch_size=B, lr=CFG["lr"], momentum_decay=CFG["beta"], temperature=CFG["T"],
                   steps_per_graph=min(100, k), perm_seed=7)
        plan = model.sgmcmc_graphs(X, Y, N_, k, **run)
        for gph, _ in plan:
            gph.launch()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        model.run_sgmcmc(X, Y, N_, k, **run)
        e1.record()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        fw, bw = step_flops(B, d, R, P, g)
        out[str(B)] = {"steps_per_s": round(k / dt, 1), "us_per_step": round(dt * 1e6 / k, 2),
                       "us_per_step_events": round(e0.elapsed_time(e1) * 1e3 / k, 2),
                       "step_mflop": round((sum(fw) + sum(bw)) / 1e6, 2),
                       "step_mfma_frac": round((sum(fw) + sum(bw)) / (dt / k) / FP32_MFMA_PEAK, 4),
                       "steps": k}
    assert torch.isfinite(model._engine.theta).all(), "b-sweep chain diverged"
    return out


def resolve_world(gpus, env, backend, device_count):
    """What this process does for `--gpus gpus`: ("run", world) — be one rank of `world` — or
    ("spawn", gpus) — start `gpus` ranks as children.  Raises SystemExit (non-zero) when the
    launcher's WORLD_SIZE disagrees with --gpus, or when nccl (RCCL, one GPU per rank) is asked for
    more ranks than visible GPUs.  `device_count` is a callable (torch.cuda.device_count does not
    initialise the GPU on this image)."""
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1, got {gpus}")
    ws = env.get("WORLD_SIZE")
    if ws is not None and int(ws) != gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={ws} from the launcher but --gpus {gpus}")
    if backend == "nccl" and gpus > 1 and device_count() < gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} with the nccl backend (one GPU per rank) but "
                         f"only {device_count()} GPU(s) visible")
    if ws is None and gpus > 1:
        return "spawn", gpus
    return "run", int(ws) if ws is not None else 1


def spawn_ranks(gpus, argv):
    """Run this script as `gpus` ranks under torch.distributed.run (127.0.0.1, a free port) and
    return its exit status; rank 0 prints the JSON line on the inherited stdout."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={gpus}", "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--steps-per-graph", type=int, default=100)
    # posterior samples scored per predictive call: the count the reference's default driver
    # collects, (total_epochs - start_sampling_epoch) / epochs_per_cycle = (5000 - 2000) / 50
    # (experiments/utils_training.py:11-16, 62-67)
    ap.add_argument("--pred-samples", type=int, default=60)
    ap.add_argument("--multi-chains", type=int, default=64)
    ap.add_argument("--full-bayes-steps", type=int, default=2000)
    ap.add_argument("--cpu-runs", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--profile-reps", type=int, default=200)
    ap.add_argument("--other-configs", type=int, default=1)
    ap.add_argument("--other-steps", type=int, default=1000)
    ap.add_argument("--b-sweep", type=int, default=1)
    ap.add_argument("--eager-calls", type=int, default=2000)
    ap.add_argument("--driver-epochs", type=int, default=6)
    args = ap.parse_args()

    # DGPRF_BENCH_BACKEND=gloo (with ranks sharing a GPU: local % device_count) rehearses the N > 1
    # path on a one-GPU box; the driver's multi-GPU runs use nccl (= RCCL), one GPU per rank
    backend = os.environ.get("DGPRF_BENCH_BACKEND", "nccl")
    what, world = resolve_world(args.gpus, os.environ, backend, torch.cuda.device_count)
    if what == "spawn":
        sys.exit(spawn_ranks(world, sys.argv[1:]))
    rank = int(os.environ.get("RANK", 0))
    local = int(os.environ.get("LOCAL_RANK", 0))
    local = local % max(1, torch.cuda.device_count()) if backend == "gloo" else local
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from dgprf import engine as E
    from dgprf import _native as N
    from dgprf.data import regression_data
    from dgprf.distributed import chain_model, rank_seed
    from dgprf.predictive import PredictiveLSE
    from likelihoods import Gaussian
    from models.regression_model import RegressionDGP

    def barrier_sync():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    N_, B = CFG["N"], CFG["B"]
    X, Y, a = regression_data(N_, CFG["D"], seed=0, device=dev)
    Xt, Yt, _ = regression_data(CFG["N_test"], CFG["D"], seed=1, device=dev, a=a)
    # one posterior: z / hyper-parameters from the rank-independent model seed on every rank,
    # the rank folded only into this chain's noise key, W init and momenta
    model = chain_model(lambda: RegressionDGP(CFG["D"], 1, n_hidden_layers=CFG["L"],
                                              n_rf=CFG["n_rf"], n_gp=CFG["n_gp"],
                                              likelihood=Gaussian(variance=CFG["variance"])),
                        2, rank)
    model.precond_update(None, N_, precond_type="identity")
    run = dict(batch_size=B, lr=CFG["lr"], momentum_decay=CFG["beta"], temperature=CFG["T"],
               steps_per_graph=args.steps_per_graph, perm_seed=rank_seed(0, rank))

    # ---------------- SGHMC steps (graph-replayed, on-device minibatching)
    # Every hipGraph the timed call replays is captured and instantiated here, the W warm-up steps
    # run, and then each timed graph is launched once (untimed) right before the clock: the timed
    # region is replays only, and its first replay does not follow a different graph (measured
    # +2.5 us/step on the driver's 20-step run when it did, scripts/diag/driver_shape.py).
    timed_plan = model.sgmcmc_graphs(X, Y, N_, args.steps, **run)
    timed_graphs = [{"steps_per_graph": gph.steps, "replays": reps} for gph, reps in timed_plan]
    if args.warmup > 0:
        model.run_sgmcmc(X, Y, N_, args.warmup, **run)
    for gph, _ in timed_plan:
        gph.launch()
    barrier_sync()
    es0, es1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    es0.record()  # the step graphs launch on this (torch's current) stream
    # exactly the replays run_sgmcmc(X, Y, N_, steps, **run) issues (the plan sgmcmc_graphs returned
    # above, resolved before the clock), without re-resolving the cached plan inside the clock
    for gph, reps in timed_plan:
        for _ in range(reps):
            gph.launch()
    es1.record()
    barrier_sync()
    t_steps = max_over_ranks(time.perf_counter() - t0)
    step_ms_dev = es0.elapsed_time(es1) / args.steps
    assert torch.isfinite(model._engine.theta).all(), "chain diverged"
    steps_per_s = world * args.steps / t_steps

    # ---------------- predictive samples (full test forward + log p + se + LSE fold)
    # The driver scores the posterior samples it has collected (utils_training.py:79-85): here the
    # chain's W at pred_samples successive SGHMC steps, scored by ONE PredictiveLSE.add_samples call
    # (dgprf_forward_samples: the pair kernel, layer 0 shared by each pair since Omega is fixed,
    # every pair in one launch, then the fold in sample order).  The one-sample launch is timed
    # beside it.
    S_pred = max(2, args.pred_samples)
    th_all = [model._engine.theta.clone()]
    for _ in range(S_pred - 1):
        model.run_sgmcmc(X, Y, N_, 1, **run)
        th_all.append(model._engine.theta.clone())
    th_all = torch.stack(th_all)  # [S, 1, w_total]
    acc = PredictiveLSE(model._engine, Xt, Yt)
    acc.add_samples(th_all)  # scratch allocation and first launch outside the clock
    acc = PredictiveLSE(model._engine, Xt, Yt)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier_sync()
    t0 = time.perf_counter()
    ev0.record()
    acc.add_samples(th_all, build=False)
    ev1.record()
    ll, rmse = acc.finalize(y_std=1.0)
    barrier_sync()
    t_pred = max_over_ranks(time.perf_counter() - t0)
    pred_kernel_ms = ev0.elapsed_time(ev1) / S_pred  # per sample (the launch + the fold)
    pred_per_s = world * S_pred / t_pred
    acc1 = PredictiveLSE(model._engine, Xt, Yt)
    acc1.add_sample(build=False)
    ev2, ev3 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    ev2.record()
    for _ in range(10):
        acc1.add_sample(build=False)
    ev3.record()
    torch.cuda.synchronize()
    single_ms = ev2.elapsed_time(ev3) / 10
    del acc1

    # ---------------- per-kernel device times (hipEvents on the launch stream) -> roofline
    eng = model._engine
    pl = eng.layout
    d, R, P, g = (list(pl.d[:3]), list(pl.n_rf[:3]), list(pl.P[:3]), list(pl.n_gp[:3]))
    prof = eng.profile_step(X, Y, B, N_, CFG["lr"], CFG["beta"], CFG["T"], reps=args.profile_reps)
    fwd_f, bwd_f = step_flops(B, d, R, P, g)
    # Per-kernel device time: the event pair around each kernel minus an empty pair recorded the
    # same way (the pair's own cost); the steady-state step time itself comes from the events over
    # the timed region (step_ms_dev), whose remainder is kernel-boundary time.
    inflow = list(prof["fwd"]) + list(prof["bwd"]) + [prof["update"]]
    att = [max(x - prof["empty"], 1e-6) for x in inflow]
    Lk = len(prof["fwd"])
    att_fwd, att_bwd, att_upd = att[:Lk], att[Lk:2 * Lk], att[2 * Lk]
    # a folded output layer (plan.fold_out) launches no forward: its F_L is formed inside its
    # backward, whose launch then carries that layer's forward FLOPs as well
    fold = int(eng.plan_ws(B)[0].fold_out)
    n_fwd = Lk - fold
    per_name = {
        "k_step_fwd": (sum(att_fwd[:n_fwd]) / n_fwd, sum(fwd_f[:n_fwd]) / n_fwd, n_fwd),
        "k_step_bwd": (sum(att_bwd) / Lk, (sum(bwd_f) + (fwd_f[-1] if fold else 0)) / Lk, Lk),
    }
    upd_bytes = 4 * pl.w_total * (pl.n_row_tiles + 2 + 2 + 2)  # gW partials + theta/mom r/w
    dom = max(per_name, key=lambda k: per_name[k][0] * per_name[k][2])
    ms_dom, fl_dom, _ = per_name[dom]
    rp_us = rocprof_avg_us(dom)
    n_dom = per_name[dom][2]
    launched = inflow[:n_fwd] + inflow[Lk:]  # the event pairs around launched kernels
    dom_pairs = inflow[:n_fwd] if dom == "k_step_fwd" else inflow[Lk:2 * Lk]
    share_us = step_ms_dev * 1e3 * sum(dom_pairs) / sum(launched) / n_dom
    live_us = ms_dom * 1e3
    # duration per launch (`achieved` / `frac`): the committed rocprofv3 kernel trace of this bench
    # (profiles/rNN/kernel_stats_bench.csv, dispatch-weighted mean over the kernel's instances), so
    # `frac` recomputes from that file; the live in-kernel span measured here (hipEvent pair on the
    # launch stream minus an empty pair) is reported beside it and must agree within 15 %
    # (tests/test_bench_profiles.py).  Without a committed trace the live span is used.
    use_us = rp_us if rp_us else live_us
    trace_step_us = None
    tr_path = os.path.join(PROFILES, "bench_under_rocprof.json")
    if rp_us and os.path.exists(tr_path):
        with open(tr_path) as fh:
            trace_step_us = json.load(fh)["roofline"]["step_us_events"]
    n_launch = 2 * len(d) + 1 - fold
    bnd_us = launch_boundary_us(dev)
    rel = os.path.relpath(PROFILES, ROOT)
    roof = {"kernel": dom, "bound": "mfma",
            "achieved": round(fl_dom / (use_us * 1e-6) / 1e12, 6),
            "peak": FP32_MFMA_PEAK / 1e12, "unit": "TFLOP/s",
            "frac": round(fl_dom / (use_us * 1e-6) / FP32_MFMA_PEAK, 8),
            "traffic": pmc_traffic(dom),
            "traffic_source": f"{rel}/pmc_traffic.json (rocprofv3 --pmc FETCH_SIZE, WRITE_SIZE "
                              "passes of this bench; bytes per launch incl. Infinity-Cache hits)",
            "avg_launch_us": round(use_us, 3),
            "duration_source": (f"{rel}/kernel_stats_bench.csv: rocprofv3 --kernel-trace --stats "
                                "of this bench, dispatch-weighted mean duration of the kernel's "
                                "instances (a traced duration also holds the dispatch's launch and "
                                "the tracer's completion signal, DESIGN.md §5)" if rp_us else
                                "live in-kernel span (no committed trace)"),
            "live_in_kernel_us": round(live_us, 3),
            "live_frac": round(fl_dom / (live_us * 1e-6) / FP32_MFMA_PEAK, 8),
            "live_in_kernel_method": "hipEvent pair around the kernel on its launch stream minus an "
                                     "empty pair (dgprf_profile_step, --profile-reps real steps): "
                                     "the span inside the kernel, without its launch boundary",
            "live_share_us": round(share_us, 3),
            "live_share_method": "the timed region's hipEvent step time split over the step's "
                                 "kernels by their event-pair times, per launch (a lower bound "
                                 "where the pairs overlap the boundaries)",
            "flops_per_launch": int(fl_dom),
            "rocprof_avg_launch_us": rp_us,
            # the tracer's own cost per dispatch: the traced duration of the step's one-thread
            # counter kernel (k_advance) in the same trace; traced - this = the in-kernel estimate
            "trace_dispatch_overhead_us": rocprof_avg_us("k_advance"),
            "rocprof_in_kernel_us": (round(rp_us - rocprof_avg_us("k_advance"), 3)
                                     if rp_us and rocprof_avg_us("k_advance") else None),
            "launch_floor": {"launches_per_step": n_launch, "boundary_us": round(bnd_us, 3),
                             "floor_us_per_step": round(n_launch * bnd_us, 3),
                             "steps_per_s_ceiling": round(1e6 / (n_launch * bnd_us), 1),
                             "method": "live: graph of 400 dependent one-element kernels replayed, "
                                       "device time per kernel (best of 5)"},
            "step_us_events": round(step_ms_dev * 1e3, 3),
            # the traced run's own step time (tracing slows every dispatch): the trace's duration
            # rescaled by plain / traced step time is what the live span is checked against
            "trace_step_us": trace_step_us,
            "rocprof_scaled_us": (round(rp_us * step_ms_dev * 1e3 / trace_step_us, 3)
                                  if rp_us and trace_step_us else None),
            "empty_pair_us": round(prof["empty"] * 1e3, 3),
            "output_layer_folded": bool(fold),
            "step_kernel_us": {"fwd": [round(x * 1e3, 3) for x in att_fwd[:n_fwd]],
                               "bwd": [round(x * 1e3, 3) for x in att_bwd],
                               "update": round(att_upd * 1e3, 3)},
            "inflow_event_us": [round(x * 1e3, 3) for x in inflow],
            "update_hbm_GBps": round(upd_bytes / (att_upd * 1e-3) / 1e9, 2),
            "regime": "latency-bound at B=200: 51.6 MFLOP/step; see DESIGN.md"}
    fp1 = pred_flops(CFG["N_test"], d, R, P, g)
    # executed per sample in a pair pass: layer 0's A = X Omega_1 once for the two samples
    fp = fp1 - CFG["N_test"] * d[0] * R[0]
    # sin + cos per RBF feature per test row (layer 0's once per pair)
    n_trans = CFG["N_test"] * (R[0] + sum(2 * r for r in R[1:]))
    roof_pred = {"kernel": "k_forward_pairs", "bound": "mfma",
                 "achieved": round(fp / (pred_kernel_ms * 1e-3) / 1e12, 4),
                 "peak": FP32_MFMA_PEAK / 1e12, "unit": "TFLOP/s",
                 "frac": round(fp / (pred_kernel_ms * 1e-3) / FP32_MFMA_PEAK, 5),
                 "traffic": pmc_traffic("k_forward_pairs"),
                 "traffic_per": f"launch ({S_pred} samples; the PMC passes run the same count)",
                 # X, Y once; per sample log p + se written and read back by the fold; the three
                 # accumulators read and written once
                 "algorithmic_bytes": int(4 * CFG["N_test"] * (CFG["D"] + 1 + 4 * S_pred + 6)),
                 "avg_us_per_sample": round(pred_kernel_ms * 1e3, 2),
                 "avg_launch_us": round(S_pred * pred_kernel_ms * 1e3, 2),
                 "rocprof_avg_launch_us": rocprof_avg_us("k_forward_pairs"),
                 "rocprof_fold_us": rocprof_avg_us("k_lse_fold_samples"),
                 "flops_per_sample": int(fp),
                 "flops_per_launch": int(S_pred * fp),
                 "flops_note": "executed FLOPs: SURVEY §8d's per-sample count minus layer 0's "
                               "X Omega_1 once per pair (one A-tile pass serves both samples)",
                 "samples_per_launch": S_pred,
                 "launch_form": "every sample pair in one launch (grid.z = pair), per-row log p "
                                "to scratch, k_lse_fold_samples folds them in sample order "
                                "(avg_launch_us: both kernels, by events)",
                 "single_sample": {"kernel": "k_forward_tiles",
                                   "us_per_sample": round(single_ms * 1e3, 2),
                                   "frac": round(fp1 / (single_ms * 1e-3) / FP32_MFMA_PEAK, 5),
                                   "rocprof_avg_launch_us": rocprof_avg_us("k_forward_tiles"),
                                   "traffic": pmc_traffic("k_forward_tiles")},
                 "transcendental_ceiling": {
                     "sin_cos_per_sample": int(n_trans), "rate_per_s": TRANS_PER_S,
                     "floor_us": round(n_trans / TRANS_PER_S * 1e6, 2),
                     "frac_of_sample_time": round(n_trans / TRANS_PER_S / (pred_kernel_ms * 1e-3), 4),
                     "rate_source": "MI355X_MICROARCH.md: v_sin_f32 / v_cos_f32 8 issue cycles per "
                                    "wave instruction, 1024 SIMDs, 2.4 GHz"}}

    # ---------------- the reference driver's per-call path (extra, not `value`)
    eager = eager_api(model, X, Y, N_, B, calls=args.eager_calls) if args.eager_calls > 0 else None

    # ---------------- the reference's driver loop end to end (extra, not `value`)
    driver = (driver_loop(dev, rank, X, Y, Xt, Yt, epochs=args.driver_epochs)
              if args.driver_epochs > 0 else None)

    # ---------------- many chains per GPU (aggregate chain-steps/s; extra, not `value`)
    multi = None
    if args.multi_chains > 1:
        spec = eng.spec
        me = E.Engine(spec, args.multi_chains, seed=rank_seed(3, rank))
        me.z.copy_(eng.z)
        me.hyp.copy_(eng.hyp)
        E.normal(None, N.RNG_W, out=me.theta)
        me.init_moments()
        me.lik_log_var_source = eng.lik_log_var_source
        me.build_omega()
        k_m = max(50, args.steps // 20)
        gph = me.graph(X, Y, B, N_, CFG["lr"], CFG["beta"], CFG["T"], 50)
        gph.launch()
        barrier_sync()
        t0 = time.perf_counter()
        for _ in range(k_m // 50):
            gph.launch()
        barrier_sync()
        t_m = max_over_ranks(time.perf_counter() - t0)
        multi = {"chains_per_gpu": args.multi_chains,
                 "chain_steps_per_s": round(world * args.multi_chains * (k_m // 50) * 50 / t_m, 1),
                 "ms_per_step_all_chains": round(t_m * 1e3 / ((k_m // 50) * 50), 4)}
        del me, gph

    # ---------------- full_bayesian=True steps (extra, not `value`): W + kernel / likelihood
    # hyper-parameters sampled, Omega/c/sigma^2 rebuilt on the device every step
    full_bayes = None
    if args.full_bayes_steps > 0:
        model.precond_update(None, N_, precond_type="identity", full_bayesian=True)
        model.run_sgmcmc(X, Y, N_, args.steps_per_graph, full_bayesian=True, **run)
        k_fb = max(args.steps_per_graph, args.full_bayes_steps // args.steps_per_graph *
                   args.steps_per_graph)
        barrier_sync()
        t0 = time.perf_counter()
        model.run_sgmcmc(X, Y, N_, k_fb, full_bayesian=True, **run)
        barrier_sync()
        t_fb = max_over_ranks(time.perf_counter() - t0)
        assert torch.isfinite(model._engine.hyp).all(), "full-Bayes chain diverged"
        full_bayes = {"steps_per_s": round(world * k_fb / t_fb, 2),
                      "us_per_step": round(t_fb * 1e6 / k_fb, 3), "steps": k_fb,
                      "sampled": "W, log_amplitude, log_inv_length_scale (ARD), lik_log_var"}

    # ---------------- BASELINE configs 3-5 at their full model shapes (extra, not `value`)
    other = {}
    if args.other_configs:
        for cfg in (3, 4, 5):
            other[f"config{cfg}"] = bench_config(cfg, dev, rank, world, barrier_sync,
                                                 max_over_ranks, args.other_steps)

    sweep = None
    if args.b_sweep:
        sweep = b_sweep(model, X, Y, N_, [(200, 2000), (1024, 1000), (8192, 400), (65536, 100)],
                        d, R, P, g)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(runs=args.cpu_runs)

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(steps_per_s, 2), "unit": "steps/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(t_steps * 1e3 / args.steps, 5), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic config 2: X~N(0,I) [1e6,8] seed 0, y=sin(Xa)+0.1eps standardized; "
                    "test [1e5,8] seed 1; random-init weights (Philox)",
            "config": {"workload": "config2: 3-layer RBF-RF DGP, n_rf=1024 (Phi 2048), g=[8,8,1], "
                                   "D=8, N=1e6, B=200, Gaussian s2=0.1, SGHMC lr=0.01 beta=0.9 T=1, "
                                   "W-only, identity preconditioner",
                       "chains_per_gpu": 1,
                       "timed_graphs": timed_graphs,
                       "timed_region": "hipGraph replays only: the graphs of "
                                       "sgmcmc_graphs(steps) (what run_sgmcmc replays), captured "
                                       "and launched once before the clock, replayed directly",
                       "parallelism": f"chain-parallel x{world} (independent chains, RCCL "
                                      "all-gather of predictive accumulators only)"},
            "predictive_samples_per_s": round(pred_per_s, 3),
            "predictive": {"n_test": CFG["N_test"], "samples": S_pred,
                           "test_loglik": round(ll, 6), "test_rmse": round(rmse, 6),
                           "ms_per_sample": round(t_pred * 1e3 / S_pred, 4)},
            "roofline": roof, "roofline_predictive": roof_pred, "cpu_baseline": cpu,
            "eager_api": eager, "driver": driver, "multi_chain": multi, "full_bayes": full_bayes, "other_configs": other or None,
            "b_sweep": sweep,
            "device": torch.cuda.get_device_name(dev),
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
