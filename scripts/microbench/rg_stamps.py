"""Diagnostic: per-segment cycle counts of the row-group backward (k_step_bwd_rg) from the
-DDGPRF_STAMPS build, config 2 at a large minibatch.

  make -C dgp-rf-mcmc_amd/csrc OUT=../../scripts/microbench/libdgprf_stamps.so EXTRA=-DDGPRF_STAMPS \
      ../../scripts/microbench/libdgprf_stamps.so
  DGPRF_LIB=scripts/microbench/libdgprf_stamps.so python scripts/microbench/rg_stamps.py [B] [rw]
Slots: 0 start, 1 after slice staging + first prologue issue, 2 first super tile's prologue barrier,
3 its compute done, 4 its end, 5 second super tile's end, 6 loop end, 7 gW stored, 14 exit.
Stamps are read only from their own buffer; nothing here is a product number.
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

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
dev = torch.device("cuda", 0)
X, Y, _ = regression_data(1_000_000, 8, 0, device=dev)
m = RegressionDGP(8, 1, n_hidden_layers=3, n_rf=1024, n_gp=[8, 8, 1], likelihood=Gaussian())
m.precond_update(None, 1_000_000, precond_type="identity")
eng = m._engine
eng.build_omega()
# through the C-ABI of the library DGPRF_LIB names (the torch op library links the product one)
pl, ws = eng.plan_ws(B)
ch = eng.chain_struct(ws)
bt = eng.batch_struct(X, Y, N.BATCH_EPOCH, iters=X.shape[0] // B, perm_seed=0)
st = eng.step_struct(0.01, 0.9, 1.0, 1_000_000)
for _ in range(20):
    N.call("dgprf_sghmc_step", ctypes.byref(pl), ctypes.byref(ch), ctypes.byref(bt),
           ctypes.byref(st), E.stream())
torch.cuda.synchronize()
lib = N.lib()
f = lib.dgprf_debug_read_rg_stamps
f.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
n = 17 * 4096 * 16
buf = (ctypes.c_ulonglong * n)()
assert f(ctypes.cast(buf, ctypes.c_void_p), n) == 0
S = np.frombuffer(buf, dtype=np.uint64).reshape(17, 4096, 16).astype(np.int64)
# row-wave kernel (k_step_bwd_rw): 0 start, 1 staged, 2+3i / 3+3i / 4+3i wave 0's row tile i start /
# tile loaded / chunks done, 11 wave 0's loop end, 12 after the barrier, 13 the last wave's loop end,
# 14 exit
RW = len(sys.argv) > 2 and sys.argv[2] == "rw"
slots = [0, 1, 2, 3, 4, 5, 6, 7, 11, 12, 14] if RW else [0, 1, 2, 3, 4, 5, 6, 7, 14]
for l in range(3):
    s = S[2 * l + 1]
    live = s[:, 0] > 0
    s = s[live]
    if not len(s):
        continue
    t0 = s[:, 0].min()
    rel = {k: s[:, k] - s[:, 0] for k in slots}
    print(f"bwd layer {l}: {live.sum()} workgroups; start spread {(s[:, 0] - t0).max()} cycles")
    for a, b in zip(slots[:-1], slots[1:]):
        d = s[:, b] - s[:, a]
        print(f"  slot {a:2d} -> {b:2d}: median {int(np.median(d)):7d}  max {int(d.max()):7d} cycles")
    if RW:
        d = s[:, 13] - s[:, 11]
        print(f"  last wave loop end - wave 0 loop end: median {int(np.median(d))}  max {int(d.max())}")
    tot = s[:, 14] - s[:, 0]
    print(f"  total median {int(np.median(tot))} max {int(tot.max())} cycles; "
          f"first start -> last end {int(s[:, 14].max() - t0)}")
