"""Diagnostic: per-wave timeline of the predictive tile kernel from the -DDGPRF_PSTAMPS build.

  make -C dgp-rf-mcmc_amd/csrc OUT=../../scripts/variants/libdgprf_pstamps.so OBJDIR=build_pst \
       EXTRA=-DDGPRF_PSTAMPS
  DGPRF_LIB=$PWD/scripts/variants/libdgprf_pstamps.so python scripts/microbench/pred_stamps.py
Reports wave lifetimes (shader cycles), per-layer cycles, waves resident per SIMD over time and the
kernel span (s_memrealtime, 100 MHz).  Diagnostics only: nothing here is a product number.
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgp-rf-mcmc_amd")]

from dgprf import _native as N  # noqa: E402
from dgprf import engine as E  # noqa: E402
from dgprf.data import regression_data  # noqa: E402
from dgprf.predictive import PredictiveLSE  # noqa: E402
from likelihoods import Gaussian  # noqa: E402
from models.regression_model import RegressionDGP  # noqa: E402

n_test = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 100_000
dev = torch.device("cuda", 0)
_, _, a = regression_data(1000, 8, seed=0, device=dev)
Xt, Yt, _ = regression_data(n_test, 8, seed=1, device=dev, a=a)
E.set_seed(2)
NL = int(sys.argv[sys.argv.index("--layers") + 1]) if "--layers" in sys.argv else 3
m = RegressionDGP(8, 1, n_hidden_layers=NL, n_rf=1024, n_gp=[8] * (NL - 1) + [1], likelihood=Gaussian())
if "--xscale" in sys.argv:  # probe: scale the test inputs (data-dependence of layer 0's time)
    Xt = Xt * float(sys.argv[sys.argv.index("--xscale") + 1])
m.precond_update(None, 1_000_000, precond_type="identity")
def _arg(name, dflt=0):
    return int(sys.argv[sys.argv.index(name) + 1]) if name in sys.argv else dflt


# placement probes: move Omega / theta by a number of floats inside a larger allocation
eng = m._engine
for nm, k in (("omega", _arg("--om-shift")), ("theta", _arg("--th-shift"))):
    if k:
        t = getattr(eng, nm)
        big = torch.empty(t.numel() + k, dtype=t.dtype, device=t.device)
        v = big[k:k + t.numel()].view(t.shape)
        v.copy_(t)
        setattr(eng, nm, v)
        print(f"{nm} moved by {k} floats", flush=True)
acc = PredictiveLSE(m._engine, Xt, Yt)
PAIRS = "--pairs" in sys.argv  # k_forward_pairs: slots 1 / 2 / 3 = after layer 0, sample 0, sample 1
for _ in range(3):
    if PAIRS:
        th = m._engine.theta
        acc.add_samples(torch.stack([th, th]))
    else:
        acc.add_sample()
torch.cuda.synchronize()
nw = (n_test + 15) // 16
nw = (nw + 15) // 16 * 16
buf = (ctypes.c_ulonglong * (nw * 8))()
lib = N.lib()
lib.dgprf_debug_read_pred_stamps.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
assert lib.dgprf_debug_read_pred_stamps(buf, nw * 8) == 0
st = np.frombuffer(buf, dtype=np.uint64).reshape(nw, 8).astype(np.int64)
st = st[st[:, 6] > 0]
rt0, rt1 = st[:, 0], st[:, 6]
t0 = rt0.min()
span_us = (rt1.max() - t0) / 100.0
life = st[:, 4 - 1] - st[:, 7]  # memtime after layer 3 - entry
lay = np.stack([st[:, 1] - st[:, 7], st[:, 2] - st[:, 1], st[:, 3] - st[:, 2]], axis=1)
print(f"waves {len(st)}  kernel span {span_us:.1f} us (realtime)")
print(f"wave lifetime cycles: median {np.median(life):.0f}  p10 {np.percentile(life, 10):.0f}  "
      f"p90 {np.percentile(life, 90):.0f}  max {life.max()}")
print("per-layer cycles (median):" if not PAIRS else
      "cycles (median) [layer 0 of the pair, sample 0 layers >= 1, sample 1 layers >= 1]:",
      [int(np.median(lay[:, i])) for i in range(3)])
print(f"wave realtime life us: median {np.median(rt1 - rt0) / 100:.1f}")
if not PAIRS:
    print("input staging cycles (entry -> rows in LDS), median:", int(np.median(st[:, 4] - st[:, 7])))
hw = st[:, 5] & 0xFFFFFFFF
xcc = st[:, 5] >> 32
simd = (hw >> 4) & 3
cu = (hw >> 8) & 15
se = (hw >> 13) & 7
key = xcc * 1000 + se * 100 + cu * 4 + simd
uk, cnt = np.unique(key, return_counts=True)
print(f"SIMDs used {len(uk)}  waves per SIMD: min {cnt.min()} median {np.median(cnt)} max {cnt.max()}")
# resident waves per SIMD over time (sampled at 20 points)
for q in np.linspace(0.05, 0.95, 10):
    t = t0 + q * (rt1.max() - t0)
    live = (rt0 <= t) & (rt1 > t)
    print(f"  t={q * span_us:6.1f} us  resident waves {live.sum():5d}  "
          f"({live.sum() / max(len(uk), 1):.2f} per SIMD)")
starts = np.sort((rt0 - t0) / 100.0)
print("start-time quantiles us:", [round(float(np.percentile(starts, p)), 1)
                                   for p in (0, 25, 50, 65, 75, 90, 100)])
early = (rt0 - t0) < 100  # started within 1 us: the first round of resident waves
for nm, sel in (("first round", early), ("later", ~early)):
    if sel.any():
        print(f"{nm}: {sel.sum()} waves, per-layer cycles median",
              [int(np.median(lay[sel, i])) for i in range(3)],
              f"life us median {np.median((rt1 - rt0)[sel]) / 100:.1f}")
# layer-1 cycles vs. entry memtime -> effective clock during layer 1 (cycles per realtime tick)
clk = (st[:, 3] - st[:, 7]) / np.maximum(rt1 - rt0, 1) / 10.0
print(f"shader GHz over wave life (median): {np.median(clk) * 1e-0:.2f}")
