"""Diagnostic: where the per-call sgmcmc_update time goes (config 2, B = 200, device batches).

  python scripts/diag/eager_layers.py [calls]

Times `calls` back-to-back calls (wall clock, one synchronize at the end) of
  (a) model.sgmcmc_update      (the reference driver's call)
  (b) Engine.step(build=False) (below the model's checks / Omega staleness test)
  (c) torch.ops.dgprf.sghmc_step_ with prebuilt arguments (the op + C-ABI + 7 launches)
  (d) (a) with the op replaced by a no-op: the Python layers alone
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgp-rf-mcmc_amd")]
from dgprf import _native as N  # noqa: E402
from dgprf import engine as E  # noqa: E402
from dgprf.data import regression_data  # noqa: E402
from likelihoods import Gaussian  # noqa: E402
from models.regression_model import RegressionDGP  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
dev = torch.device("cuda", 0)
X, Y, _ = regression_data(1_000_000, 8, seed=0, device=dev)
E.set_seed(3)
m = RegressionDGP(8, 1, n_hidden_layers=3, n_rf=1024, n_gp=[8, 8, 1],
                  likelihood=Gaussian(variance=0.1))
m.precond_update(None, 1_000_000, precond_type="identity")
eng = m._engine
xs = [X[i * 200:(i + 1) * 200] for i in range(50)]
ys = [Y[i * 200:(i + 1) * 200] for i in range(50)]


def timed(fn):
    for i in range(50):
        fn(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(calls):
        fn(i % 50)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e6 / calls


a = timed(lambda i: m.sgmcmc_update(xs[i], ys[i], 1_000_000, lr=0.01, momentum_decay=0.9))
b = timed(lambda i: eng.step(xs[i], ys[i], 1_000_000, 0.01, 0.9, 1.0, build=False))
pl, ws, _, _, _, _, ps = eng._op_batch(xs[0], ys[0], None, N.BATCH_DIRECT, None, 0)
pt = eng._plan_t(pl)
op = E.ops().sghmc_step_
args = lambda i: (pt, eng.theta, eng.mom, eng.omega, eng.der, eng.mass, ws, eng.step_ctr,
                  E._i64(eng.seed), xs[i], ys[i], int(N.BATCH_DIRECT), 0, ps, None, 0.01, 0.9, 1.0,
                  1e6, False, None, None, False, eng.z, eng.hyp, eng.hmom, eng.hmass, None, None)
pre = [args(i) for i in range(50)]
c = timed(lambda i: op(*pre[i]))


class _NoOp:
    def __getattr__(self, name):
        return lambda *a, **k: None


real = E.ops
E.ops = lambda: _NoOp()
d = timed(lambda i: m.sgmcmc_update(xs[i], ys[i], 1_000_000, lr=0.01, momentum_decay=0.9))
E.ops = real
print(f"us per call: (a) sgmcmc_update {a:.1f}  (b) Engine.step {b:.1f}  (c) op only {c:.1f}  "
      f"(d) python layers only {d:.1f}", flush=True)

# host issue time vs device time of the op-only loop: host-bound when the issue time per call
# matches the wall time per call
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize()
t0 = time.perf_counter()
e0.record()
for i in range(calls):
    op(*pre[i % 50])
e1.record()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"op-only: host issue {(t1 - t0) * 1e6 / calls:.1f} us/call, wall {(t2 - t0) * 1e6 / calls:.1f}, "
      f"device (events) {e0.elapsed_time(e1) * 1e3 / calls:.1f}", flush=True)

# the same op-only loop on a non-default stream (torch's default stream is HIP's null stream)
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    for i in range(50):
        op(*pre[i % 50])
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record()
    for i in range(calls):
        op(*pre[i % 50])
    e1.record()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
print(f"op-only on a side stream: host issue {(t1 - t0) * 1e6 / calls:.1f} us/call, wall "
      f"{(t2 - t0) * 1e6 / calls:.1f}, device (events) {e0.elapsed_time(e1) * 1e3 / calls:.1f}", flush=True)
