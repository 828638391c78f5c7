"""Diagnostic: per-segment cycle counts of the step kernels from the -DDGPRF_STAMPS build.

  make -C dgp-rf-mcmc_amd/csrc OUT=../../scripts/microbench/libdgprf_stamps.so EXTRA=-DDGPRF_STAMPS
  DGPRF_LIB=scripts/microbench/libdgprf_stamps.so python scripts/microbench/stamps.py
Stamps are read only from their own buffer; nothing here is a product number (stamps serialise).
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
from likelihoods import Gaussian  # noqa: E402
from models.regression_model import RegressionDGP  # noqa: E402

SLOTS = 16
dev = torch.device("cuda", 0)
CFG = 5 if "--config5" in sys.argv else (4 if "--config4" in sys.argv else 2)
if CFG == 4:  # config 4: 4 x RBF, n_rf 4096, g [30, 30, 30, 10], 784 inputs, softmax
    from dgprf.data import CONFIGS, classification_data  # noqa: E402
    from likelihoods import Softmax  # noqa: E402
    from models.dgp import DGP_RF  # noqa: E402
    c = CONFIGS[4]
    X, Y = classification_data(c["n"], c["d_in"], c["d_out"], seed=0, device=dev)
    m = DGP_RF(c["d_in"], c["d_out"], n_hidden_layers=len(c["kinds"]), n_rf=c["n_rf"],
               n_gp=c["n_gp"], likelihood=Softmax(), kernel_type_list=c["kinds"])
elif CFG == 5:  # config 5: L=5 mixed RBF/ARC, n_rf=8192, g=16
    X, Y, _ = regression_data(1_000_000, 16, 0, device=dev)
    m = RegressionDGP(16, 1, n_hidden_layers=5, n_rf=8192, n_gp=[16, 16, 16, 16, 1],
                      likelihood=Gaussian(), kernel_type_list=["RBF", "ARC", "RBF", "ARC", "RBF"])
else:
    X, Y, _ = regression_data(1_000_000, 8, 0, device=dev)
    m = RegressionDGP(8, 1, n_hidden_layers=3, n_rf=1024, n_gp=[8, 8, 1], likelihood=Gaussian())
FB = "--full-bayes" in sys.argv  # full_bayesian=True steps; hyper workgroups reported apart
NDATA = X.shape[0]
m.precond_update(None, NDATA, precond_type="identity", full_bayesian=FB)
eng = m._engine
lib = N.lib()
for _ in range(50):
    eng.step(X, Y, NDATA, 0.01, 0.9, 1.0, batch_size=200, mode=2, full_bayes=FB)
torch.cuda.synchronize()
lib.dgprf_debug_clear_stamps()
for _ in range(3):
    eng.step(X, Y, NDATA, 0.01, 0.9, 1.0, batch_size=200, mode=2, full_bayes=FB)
torch.cuda.synchronize()
n = 17 * 4096 * SLOTS
buf = (ctypes.c_ulonglong * n)()
assert lib.dgprf_debug_read_stamps(buf, n) == 0
S = np.frombuffer(buf, dtype=np.uint64).reshape(17, 4096, SLOTS).astype(np.int64)
# the per-tile forward / backward kernels stamp into the launcher's buffer (a.stamps)
buf2 = (ctypes.c_ulonglong * n)()
lib.dgprf_debug_read_rg_stamps.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
if lib.dgprf_debug_read_rg_stamps(buf2, n) == 0:
    S2 = np.frombuffer(buf2, dtype=np.uint64).reshape(17, 4096, SLOTS).astype(np.int64)
    S = np.where(S2 > 0, S2, S)
Lm = m.n_hidden_layers
names = {2 * l: f"fwd{l}" for l in range(Lm)}
names.update({2 * l + 1: f"bwd{l}" for l in range(Lm)})
names[16] = "update"
order = [2 * l for l in range(Lm)] + [2 * l + 1 for l in reversed(range(Lm))] + [16]
if FB:  # the update kernel's first workgroups are the hyper ones (one per 1024 Omega elements + 1)
    pl = eng.layout
    n_hyp = sum((pl.d[l] * pl.n_rf[l] + 1023) // 1024 for l in range(eng.L)) + 1
    S = np.concatenate([S, S[16:17]], axis=0)
    S[17, n_hyp:] = 0
    S[16, :n_hyp] = 0
    names[17] = "hyper"
    order.append(17)
t0_all = []
for k in order:
    st = S[k]
    valid = (st[:, 0] > 0) & (st[:, 14] > 0)
    st = st[valid]
    if len(st) == 0:
        continue
    real0, real_end = st[:, 15], st[:, 13]
    cyc = st[:, 14] - st[:, 0]
    freq = cyc / np.maximum(real_end - real0, 1) * 100e6
    segs = []
    marks = [i for i in range(0, 13) if (st[:, i] > 0).all()] + [14]
    if False:  # placement (needs DGPRF_STAMP_HWID in the kernel): HW_ID (simd [5:4], cu [11:8], sh [12], se [15:13]) | XCC << 32
        hw = st[:, 8:12]
        simd = (hw >> 4) & 3
        cu_key = ((hw[:, 0] >> 32) << 16) | (((hw[:, 0] >> 13) & 7) << 8) | (((hw[:, 0] >> 12) & 1) << 4) | ((hw[:, 0] >> 8) & 15)
        uniq, cnt = np.unique(cu_key, return_counts=True)
        simds_distinct = np.array([len(set(r)) for r in simd])
        print(f"  placement {names[k]}: {len(uniq)} distinct CUs for {len(st)} WGs, WGs/CU max {cnt.max()}, "
              f"distinct SIMDs per WG min {simds_distinct.min()} median {np.median(simds_distinct)}")
    marks.sort(key=lambda i: np.median(st[:, i] - st[:, 0]))  # program order
    for a, b in zip(marks[:-1], marks[1:]):
        segs.append(f"{a}->{b}: {np.median(st[:, b] - st[:, a]):.0f}")
    span = (real_end.max() - real0.min()) * 10
    skew = (real0.max() - real0.min()) * 10
    print(f"{names[k]:7s} WGs={len(st):4d} clock~{np.median(freq) / 1e9:.2f}GHz  "
          f"median cycles [{', '.join(segs)}]  total {np.median(cyc):.0f}  "
          f"span {span:.0f} ns  start-skew {skew:.0f} ns")
    t0_all.append((names[k], real0.min(), real_end.max()))
print("kernel-to-kernel (first WG start of next - last WG end of previous), ns:")
for (a, s0, e0), (b, s1, e1) in zip(t0_all[:-1], t0_all[1:]):
    print(f"  {a} -> {b}: {(s1 - e0) * 10}")
