"""Device-resident chain engine: packed HBM state + the libdgprf.so calls of the hot path.

One Engine holds the state the reference spreads over tf.Variables and their ad-hoc attributes
(models/dgp.py:66-68, 208-216, 235-296):
  theta [C, w_total]   every W_l of every chain, packed (GPLayer.W views into it)
  mom   [C, w_total]   SGHMC momenta (`param.moments`)
  mass  [C, L]         preconditioner M per W_l (`param.M`)
  z, omega [omega_total], hyp [hyp_total], der [der_total]   RF frequencies / kernel hyper-params
  step  int64[1]       device step counter (Philox counter, minibatch position, schedule)
Workspaces are sized per minibatch size B and cached.  Everything runs on torch's current HIP
stream; torch only provides memory, streams and collectives.
"""
import ctypes
import math
import weakref

import numpy as np
import torch

from . import _native as N

_F32 = torch.float32


def device():
    """The HIP device the engine runs on.  There is no CPU fallback."""
    if not torch.cuda.is_available():
        raise RuntimeError(
            "dgprf requires an AMD Instinct (gfx950) HIP device; none is visible. "
            "The DGP-RF hot path has no CPU fallback.")
    return torch.device("cuda", torch.cuda.current_device())


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def as_device(x, dev, dtype=_F32):
    """Host array / tensor -> contiguous fp32 device tensor (no copy if already there)."""
    if not torch.is_tensor(x):
        x = torch.as_tensor(x)
    return x.to(device=dev, dtype=dtype).contiguous()


class HostStage:
    """Per-call host batches (numpy, or CPU tensors) -> device, as the reference's driver loop
    feeds them (experiments/utils_training.py:45-61): X and Y are packed into one slot of a ring
    of pinned host buffers and sent with ONE asynchronous H2D copy into the matching device slot,
    instead of two pageable copies that each block the host until the GPU drained the previous
    step.  A slot (pinned and device buffer) is rewritten only after the event recorded behind
    the op that read it completed (release(); behind the copy if no op followed), so the ring is
    safe when calls alternate streams too."""
    SLOTS = 4

    def __init__(self, dev):
        self.dev = dev
        self.cap = 0
        self.k = 0

    def _grow(self, n):
        self.cap = max(int(n), 2 * self.cap, 4096)
        self.host = [torch.empty(self.cap, dtype=_F32, pin_memory=True) for _ in range(self.SLOTS)]
        self.host_np = [h.numpy() for h in self.host]
        self.devb = [torch.empty(self.cap, dtype=_F32, device=self.dev) for _ in range(self.SLOTS)]
        self.ev = [torch.cuda.Event() for _ in range(self.SLOTS)]
        self.used = [False] * self.SLOTS
        self.views = {}  # (slot, X shape, Y shape) -> host / device views of that slot

    def _views(self, i, xs, ys):
        key = (i, xs, ys)
        v = self.views.get(key)
        if v is None:
            if len(self.views) >= 64:  # many distinct batch shapes: start over
                self.views.clear()
            nx, ny = math.prod(xs), math.prod(ys)
            h, d = self.host_np[i], self.devb[i]
            v = (h[:nx].reshape(xs), h[nx:nx + ny].reshape(ys), self.host[i][:nx + ny],
                 d[:nx + ny], d[:nx].view(xs), d[nx:nx + ny].view(ys))
            self.views[key] = v
        return v

    @staticmethod
    def _host_array(t):
        if not torch.is_tensor(t):
            return np.asarray(t)
        t = t.detach()
        return (t.float() if t.dtype == torch.bfloat16 else t).numpy()

    def put(self, X, Y):
        Xn, Yn = self._host_array(X), self._host_array(Y)
        if Xn.ndim != 2:
            raise ValueError(f"X must be 2-D, got shape {Xn.shape}")
        if Xn.size + Yn.size > self.cap:
            if self.cap:
                torch.cuda.synchronize(self.dev)  # the old slots may still be in flight
            self._grow(Xn.size + Yn.size)
        i = self.k % self.SLOTS
        self.k += 1
        if self.used[i]:
            self.ev[i].synchronize()
        hx, hy, hs, ds, dx, dy = self._views(i, Xn.shape, Yn.shape)
        np.copyto(hx, Xn, casting="unsafe")
        np.copyto(hy, Yn, casting="unsafe")
        ds.copy_(hs, non_blocking=True)  # on the device's current stream, like the op
        self.ev[i].record(torch.cuda.current_stream(self.dev))
        self.used[i] = True
        self.last = i
        return dx, dy

    def release(self):
        """After the op that read the last slot was enqueued: its event now covers that op."""
        self.ev[self.last].record(torch.cuda.current_stream(self.dev))


def ops():
    """torch.ops.dgprf — the hot-path entry points registered with torch's dispatcher
    (libdgprf_torch.so over the C-ABI).  Raises if the extension is not built."""
    return N.torch_ops()


def _i64(u):
    """A uint64 key / seed as the int64 a torch op schema carries (same bits)."""
    u = int(u) & 0xFFFFFFFFFFFFFFFF
    return u - (1 << 64) if u >= (1 << 63) else u


# ------------------------------------------------------------------ global Philox stream state
class _RNG:
    """Replacement of TF's global generator: key = seed, one fresh subsequence per draw."""
    seed = 0x5EED_D6F5
    sub = 0


def set_seed(seed):
    _RNG.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    _RNG.sub = 0


def next_subsequence():
    s = _RNG.sub
    _RNG.sub += 1
    return s


def engine_key():
    """A fresh Philox key for a new Engine: the global seed mixed with the next subsequence
    (splitmix64 finaliser), so two models built in one process draw independent step noise — as
    the reference's tf.random.normal, whose global stream moves on between models
    (models/dgp.py:210-212) — while staying reproducible under set_seed."""
    x = (_RNG.seed + 0x9E3779B97F4A7C15 * (next_subsequence() + 1)) & 0xFFFFFFFFFFFFFFFF
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return x ^ (x >> 31)


def normal(shape, purpose, dev=None, out=None):
    """N(0,1) tensor drawn on the device by dgprf_philox_normal."""
    dev = dev or device()
    if out is None:
        out = torch.empty(shape, dtype=_F32, device=dev)
    N.call("dgprf_philox_normal", ptr(out), out.numel(), _RNG.seed, next_subsequence(),
           int(purpose), stream())
    return out


# ------------------------------------------------------------------ spec
class ModelSpec:
    """Static shape of a DGP_RF (the constructor arguments of models/dgp.py:9-52)."""

    def __init__(self, d_in, d_out, kinds, n_rf, n_gp, input_cat=False, likelihood=N.LIK_GAUSSIAN,
                 hyp_flags=N.HYP_KERNEL | N.HYP_LIK, ard=None):
        self.d_in, self.d_out = int(d_in), int(d_out)
        self.kinds = [int(k) for k in kinds]
        self.n_rf = [int(r) for r in n_rf]
        self.n_gp = [int(g) for g in n_gp]
        self.input_cat = bool(input_cat)
        self.likelihood = int(likelihood)
        self.L = len(self.kinds)
        # full_bayesian=True: which hyper-parameter groups are trainable, ARD per layer
        self.hyp_flags = int(hyp_flags)
        self.ard = [1] * self.L if ard is None else [int(bool(a)) for a in ard]

    def plan(self, batch=1, n_chains=1, hyp_per_chain=False):
        return N.make_plan(self.d_in, self.d_out, self.kinds, self.n_rf, self.n_gp,
                           self.input_cat, self.likelihood, batch, n_chains, self.hyp_flags,
                           hyp_per_chain, self.ard)


class _A1Entry:
    """One resident first-layer projection: the dataset tensor it was computed from (weakly held,
    so the entry cannot outlive it or be matched by another tensor at the same address), its buffer
    and the Omega_1 state it reflects."""
    __slots__ = ("xref", "buf", "okey", "__weakref__")

    def __init__(self, X, buf, okey):
        self.xref = weakref.ref(X)
        self.buf = buf
        self.okey = okey


def _a1_drop(eng_ref, key, ent_ref):
    """weakref.finalize callback of a dataset tensor: forget its projection (if still cached)."""
    eng, ent = eng_ref(), ent_ref()
    if eng is not None and ent is not None and eng._a1_cache.get(key) is ent:
        del eng._a1_cache[key]


class Engine:
    MAX_GRAPHS = 8  # instantiated step graphs kept per engine (LRU)
    A1_MAX_BYTES = 8 << 30  # resident first-layer projections (dataset_a1) larger than this: GEMM
    A1_MAX_ENTRIES = 4  # resident projections kept per engine (LRU; graphs keep their own alive)

    def __init__(self, spec, n_chains=1, dev=None, seed=None, per_chain_hyp=None):
        """per_chain_hyp: every chain owns its kernel / likelihood hyper-parameters (and Omega),
        needed to sample them with full_bayesian=True across several chains; default: only when
        C == 1 (where it changes nothing), i.e. C > 1 chains share one hyper-parameter set."""
        self.spec = spec
        self.C = int(n_chains)
        self.dev = dev or device()
        self.per_chain_hyp = (self.C == 1) if per_chain_hyp is None else bool(per_chain_hyp)
        self.layout = spec.plan(1, self.C, self.per_chain_hyp)
        pl = self.layout
        self.L = spec.L
        f = lambda n: torch.zeros(int(n), dtype=_F32, device=self.dev)
        Ch = self.C if self.per_chain_hyp else 1
        self.theta = torch.zeros(self.C, pl.w_total, dtype=_F32, device=self.dev)
        self.mom = torch.zeros(self.C, pl.w_total, dtype=_F32, device=self.dev)
        self.mass = torch.ones(self.C, self.L, dtype=_F32, device=self.dev)
        self.z = f(max(pl.omega_total, 1))
        # chain 0 first: the views below address chain 0 (the reference's single model)
        self.omega = f(max(pl.omega_total, 1) * Ch)
        self.hyp = f(pl.hyp_total * Ch)
        self.der = f(pl.der_total * Ch)
        # full_bayesian=True: hyper-parameter momenta (hyp layout) and masses (N.HMASS slots)
        self.hmom = torch.zeros(self.C, pl.hyp_total, dtype=_F32, device=self.dev)
        self.hmass = torch.ones(self.C, N.HMASS, dtype=_F32, device=self.dev)
        self.hyper_moments_ready = False
        self.step_ctr = torch.zeros(1, dtype=torch.int64, device=self.dev)
        self.seed = engine_key() if seed is None else int(seed)
        self.lik_log_var_source = None  # callable -> device scalar tensor (Gaussian likelihood)
        self._ws = {}
        self._graphs = {}
        self._fwd_scratch = None
        self._plan_tensors = {}
        self.moments_ready = False
        # wide first layer (d_1 > 32): X Omega_1 of a whole dataset / test set kept resident in HBM
        # (dataset_a1), so steps gather their rows and predictive samples share it instead of
        # running the A_1 GEMM; recomputed when Omega_1 may have changed (hyper_epoch counts device
        # full-Bayes runs, whose hyper-parameter writes torch's version counters do not see)
        self.resident_a1 = True
        self.hyper_epoch = 0
        self._a1_cache = {}
        self._stage = None  # HostStage for per-call host batches
        self._staged = False  # the current op's batch came through it (release after the op)

    # ---------------------------------------------------------------- views
    def W_view(self, l, chain=0):
        pl = self.layout
        o, P, g = pl.w_off[l], pl.P[l], pl.n_gp[l]
        return self.theta[chain, o:o + P * g].view(P, g)

    def mom_view(self, l, chain=0):
        pl = self.layout
        o, P, g = pl.w_off[l], pl.P[l], pl.n_gp[l]
        return self.mom[chain, o:o + P * g].view(P, g)

    def z_view(self, l):
        pl = self.layout
        o, d, R = pl.omega_off[l], pl.d[l], pl.n_rf[l]
        return self.z[o:o + d * R].view(d, R)

    def omega_view(self, l):
        pl = self.layout
        o, d, R = pl.omega_off[l], pl.d[l], pl.n_rf[l]
        return self.omega[o:o + d * R].view(d, R)

    def log_amp_view(self, l):
        return self.hyp[l:l + 1].view(())

    def lik_log_var_view(self):
        return self.hyp[self.L:self.L + 1].view(())

    def lis_view(self, l):
        o = self.layout.lis_off[l]
        return self.hyp[o:o + self.layout.d[l]]

    def mean_view(self, l):
        o = self.layout.mean_off[l]
        return self.hyp[o:o + self.layout.d[l]]

    def c_view(self, l):
        return self.der[l:l + 1]

    # ---------------------------------------------------------------- init draws
    def draw_init(self):
        """z ~ N(0,1), W ~ N(0,1) (layers/rf_layers.py:22, layers/GP_weight_layers.py:9)."""
        normal(None, N.RNG_Z, out=self.z)
        normal(None, N.RNG_W, out=self.theta)
        for l in range(self.L):
            self.lis_view(l).fill_(-0.5 * math.log(self.layout.d[l]))  # kernels/RBF.py:16-17,40
        self.invalidate_omega()

    def invalidate_omega(self):
        """Forget the last Omega build: a native write to z or hyp (through a raw pointer) does not
        bump torch's version counters, which build_omega_if_stale reads."""
        self._omega_built_key = None

    def init_moments(self, hyper=False):
        """param.M = 1, param.moments ~ N(0,1) (models/dgp.py:235-240); hyper=True also for the
        kernel / likelihood hyper-parameters (full_bayesian=True, vars = trainable_variables)."""
        self.mass.fill_(1.0)
        normal(None, N.RNG_MOMENTS, out=self.mom)
        self.moments_ready = True
        if hyper:
            self.init_hyper_moments()

    def init_hyper_moments(self):
        self.hmass.fill_(1.0)
        normal(None, N.RNG_MOMENTS, out=self.hmom)
        self.hyper_moments_ready = True

    def hyp_chain(self, chain):
        """[hyp_total] hyper-parameters of `chain` (the shared set when not per chain)."""
        pl = self.layout
        c = chain if self.per_chain_hyp else 0
        return self.hyp[c * pl.hyp_total:(c + 1) * pl.hyp_total]

    # ---------------------------------------------------------------- checkpoint / resume
    _STATE = ("theta", "mom", "mass", "z", "hyp", "hmom", "hmass", "step_ctr")

    def state_arrays(self):
        """The chain state as host arrays (SURVEY §5 checkpoint / resume): every tensor a step
        reads or writes — W (theta), momenta, masses, z, hyper-parameters and their momenta /
        masses, the device step counter (Philox counter, minibatch position, schedule clock) —
        plus the engine's Philox key and the moment flags.  Omega / c / sigma^2 are derived (rebuilt
        from z and hyp on load)."""
        out = {k: getattr(self, k).detach().cpu().numpy() for k in self._STATE}
        out["seed"] = np.array([self.seed], dtype=np.uint64)
        out["flags"] = np.array([self.C, int(self.per_chain_hyp), int(self.moments_ready),
                                 int(self.hyper_moments_ready)], dtype=np.int64)
        return out

    def load_state_arrays(self, st):
        """Inverse of state_arrays on an engine of the same spec and chain count."""
        C, pch, mr, hmr = (int(x) for x in st["flags"])
        if C != self.C or bool(pch) != self.per_chain_hyp:
            raise ValueError(f"checkpoint of {C} chains (per_chain_hyp={bool(pch)}) does not match "
                             f"this engine ({self.C}, {self.per_chain_hyp})")
        for k in self._STATE:
            t = getattr(self, k)
            a = torch.as_tensor(np.asarray(st[k]))
            if tuple(a.shape) != tuple(t.shape) or a.dtype != t.dtype:
                raise ValueError(f"checkpoint field {k}: {tuple(a.shape)} {a.dtype}, engine has "
                                 f"{tuple(t.shape)} {t.dtype}")
            t.copy_(a.to(t.device))
        self.seed = int(np.asarray(st["seed"], dtype=np.uint64)[0])
        self.moments_ready, self.hyper_moments_ready = bool(mr), bool(hmr)
        # captured graphs hold the old Philox key (chain_struct.seed at capture) and resident
        # projections the old Omega_1: neither may be replayed / read after a load
        self.drop_graphs()
        self._a1_cache.clear()
        self.invalidate_omega()
        self.build_omega()

    def drop_graphs(self):
        """Destroy every cached step graph (after the stream drained: replays are asynchronous)."""
        if self._graphs:
            torch.cuda.current_stream(self.dev).synchronize()
            self._graphs.clear()

    # ---------------------------------------------------------------- per-B plans
    def plan_ws(self, B, fresh_z=0, full_bayes=False):
        """(plan, zero-filled workspace) for minibatch size B; fresh_z = bit mask of the layers
        that draw fresh z every step on the device (random_fixed=False, graph steps).
        full_bayes: a plan whose backward fits full_bayesian=True steps — when B > 256 and some
        layer does not fit the full-Bayes row-group layout (rg_full_bayes == 0), the per-row-tile
        backward (plan.bwd_tiles), sized for one gW partial row per 16-row tile."""
        if full_bayes:
            pl, ws = self.plan_ws(B, fresh_z)
            if pl.rt_per_group == 1 or pl.rg_full_bayes:
                return pl, ws
        key = (int(B), int(fresh_z), bool(full_bayes))
        if key not in self._ws:
            pl = self.spec.plan(key[0], self.C, self.per_chain_hyp)
            # fresh z layers; a forward path pinned by set_forward_path also pins the step's
            # all-layer forward (large minibatches)
            if fresh_z or full_bayes or self.layout.fwd_path != N.FWD_AUTO:
                pl.fresh_z = key[1]
                pl.bwd_tiles = int(key[2])
                pl.fwd_path = self.layout.fwd_path
                pl.agemm_chunk_rows = self.layout.agemm_chunk_rows
                N.call("dgprf_plan_init", ctypes.byref(pl))
            ws = torch.zeros(max(pl.ws_total, 4), dtype=_F32, device=self.dev)
            self._ws[key] = (pl, ws)
        return self._ws[key]

    def chain_struct(self, ws, omega=None, z=None):
        c = N.Chain()
        c.theta = self.theta.data_ptr()
        c.mom = self.mom.data_ptr()
        c.omega = (self.omega if omega is None else omega).data_ptr()
        c.der = self.der.data_ptr()
        c.mass = self.mass.data_ptr()
        c.z = (self.z if z is None else z).data_ptr()
        c.hyp = self.hyp.data_ptr()
        c.hmom = self.hmom.data_ptr()
        c.hmass = self.hmass.data_ptr()
        c.ws = ws.data_ptr()
        c.step = self.step_ctr.data_ptr()
        c.seed = self.seed
        return c

    @staticmethod
    def batch_struct(X, Y, mode=N.BATCH_DIRECT, idx=None, iters=0, perm_seed=0):
        b = N.Batch()
        b.X, b.Y = X.data_ptr(), Y.data_ptr()
        b.idx = idx.data_ptr() if idx is not None else None
        b.n_data = X.shape[0]
        b.y_cols = Y.shape[1] if Y.dim() == 2 else 1
        b.mode = mode
        b.iters_per_epoch = int(iters)
        b.perm_seed = int(perm_seed)
        return b

    @staticmethod
    def step_struct(lr, beta, T, data_size, resample=False, schedule=N.SCHED_CONST,
                    start_step=0, cycle_length=1, resample_head=False, xi=None, xi_resample=None,
                    step_offset=0, full_bayes=False, xi_hyp=None, xi_hyp_resample=None):
        s = N.Step()
        s.lr, s.momentum_decay, s.temperature = float(lr), float(beta), float(T)
        s.data_size = float(data_size)
        s.resample_moments = int(bool(resample))
        s.schedule = int(schedule)
        s.step_offset = int(step_offset)
        s.grad_only = 0
        s.start_step, s.cycle_length = int(start_step), int(cycle_length)
        s.resample_in_cycle_head = int(bool(resample_head))
        s.xi = xi.data_ptr() if xi is not None else None
        s.xi_resample = xi_resample.data_ptr() if xi_resample is not None else None
        s.full_bayes = int(bool(full_bayes))
        s.xi_hyp = xi_hyp.data_ptr() if xi_hyp is not None else None
        s.xi_hyp_resample = xi_hyp_resample.data_ptr() if xi_hyp_resample is not None else None
        return s

    # ---------------------------------------------------------------- hyper-params
    def build_omega(self, z=None, omega=None):
        """Omega, c_l and sigma^2 from z / hyp (dgprf_omega_build); z/omega may be overridden
        (fresh z of layers with random_fixed=False, layers/rf_layers.py:39-41)."""
        if self.lik_log_var_source is not None:
            src = self.lik_log_var_source()
            if src is not None:
                self.lik_log_var_view().copy_(src.detach().reshape(()))
        N.call("dgprf_omega_build", ctypes.byref(self.layout),
               ptr(self.z if z is None else z), ptr(self.hyp),
               ptr(self.omega if omega is None else omega), ptr(self.der), stream())
        if z is None and omega is None:
            self._omega_built_key = self._omega_key()

    def _omega_key(self):
        """What Omega / c / sigma^2 are built from, as seen by torch: the z and hyp buffers and
        their version counters (every in-place write through them or their views — the kernel
        parameter views, an optimizer's sub_ — bumps the counter).  Device-side full-Bayes steps
        rewrite hyp and rebuild Omega together, so they leave the pair consistent."""
        return (self.z.data_ptr(), self.z._version, self.hyp.data_ptr(), self.hyp._version)

    def build_omega_if_stale(self):
        """build_omega() unless nothing it reads changed since the last full build."""
        if self.lik_log_var_source is not None:
            src = self.lik_log_var_source()
            if src is not None and src.data_ptr() != self.lik_log_var_view().data_ptr():
                self.build_omega()  # a separate source tensor: copy it in every time
                return True
        if getattr(self, "_omega_built_key", None) == self._omega_key():
            return False
        self.build_omega()
        return True

    def dataset_a1(self, X):
        """X Omega_1 for every row of X ([align64(n), n_rf[0]], rows past n zero), resident in HBM
        and cached per (X, Omega_1 state) — the first-layer projection of the reference's
        `tf.matmul(x, self.Omega)` (layers/rf_layers.py:42) for a wide first layer (d_1 > 32),
        computed once by the hand-written MFMA GEMM (dgprf_rf_project) instead of per minibatch /
        per posterior sample.  None when the layer is not wide, Omega_1 is per chain, or the
        projection would exceed A1_MAX_BYTES.  Call after Omega is built.

        An entry belongs to the X tensor object it was computed from (held by a weak reference and
        dropped when X is freed), so another dataset later placed at the same address by the
        caching allocator is projected afresh; at most A1_MAX_ENTRIES are kept (LRU)."""
        pl = self.layout
        if pl.a0_off < 0 or not self.resident_a1 or (self.per_chain_hyp and self.C > 1):
            return None
        n, R0 = int(X.shape[0]), int(pl.n_rf[0])
        rows = (n + 63) // 64 * 64
        if rows * R0 * 4 > self.A1_MAX_BYTES or R0 % 4:
            return None
        key = (id(X), X.data_ptr(), tuple(X.shape))
        okey = (X._version, self._omega_key(), self.hyper_epoch)
        ent = self._a1_cache.pop(key, None)
        if ent is not None and ent.xref() is not X:
            ent = None  # a dead tensor's entry (its finaliser has not run yet)
        if ent is None or ent.okey != okey:
            buf = ent.buf if ent is not None else torch.zeros(rows, R0, dtype=_F32, device=self.dev)
            self.rf_project(X, self.omega_view(0), out=buf[:n])
            if ent is None:
                ent = _A1Entry(X, buf, okey)
                weakref.finalize(X, _a1_drop, weakref.ref(self), key, weakref.ref(ent))
            ent.okey = okey
        self._a1_cache[key] = ent  # most recently used last
        while len(self._a1_cache) > self.A1_MAX_ENTRIES:
            self._a1_cache.pop(next(iter(self._a1_cache)))
        return ent.buf

    def invalidate_a1(self):
        """Mark every resident projection stale: the next dataset_a1 recomputes it into the same
        buffer (so graphs holding that buffer stay valid) — e.g. to time the projection inside a
        measured region."""
        for ent in self._a1_cache.values():
            ent.okey = None

    # ---------------------------------------------------------------- hot path
    def _prep_batch(self, X, Y, stage=False):
        """stage: X, Y are one call's batch (never a dataset a graph keeps): host arrays go through
        the pinned HostStage ring"""
        host = lambda t: not torch.is_tensor(t) or t.device.type == "cpu"
        if stage and host(X) and host(Y) and self.dev.type == "cuda":
            if self._stage is None:
                self._stage = HostStage(self.dev)
            X, Y = self._stage.put(X, Y)
            self._staged = True
        else:
            X = as_device(X, self.dev)
            Y = as_device(Y, self.dev)
        if X.dim() != 2 or X.shape[1] != self.spec.d_in:
            raise ValueError(f"X must be [B, {self.spec.d_in}], got {tuple(X.shape)}")
        if Y.dim() == 1:
            Y = Y[:, None]
        if Y.shape[0] != X.shape[0]:
            raise ValueError("X and Y must have the same number of rows")
        return X, Y

    def _batch(self, X, Y, batch_size, mode, idx, perm_seed):
        """(plan, ws, Batch struct, keep-alive) for a DIRECT batch (X, Y are the batch) or an
        INDEXED / EPOCH minibatch of batch_size rows drawn from the dataset (X, Y)."""
        X, Y = self._prep_batch(X, Y)
        B = X.shape[0] if mode == N.BATCH_DIRECT else int(batch_size)
        pl, ws = self.plan_ws(B)
        if idx is not None:
            idx = torch.as_tensor(idx).to(device=self.dev, dtype=torch.int32).contiguous()
        iters = X.shape[0] // B if mode == N.BATCH_EPOCH else 0
        bt = self.batch_struct(X, Y, mode, idx, iters, perm_seed)
        return pl, ws, bt, (X, Y, idx)

    def _check_full_bayes(self):
        if not self.hyper_moments_ready:
            raise AssertionError("Trainable Params do not have attr moments!")  # dgp.py:208
        if self.C > 1 and not self.per_chain_hyp:
            raise ValueError("full_bayesian=True with several chains needs per_chain_hyp=True")

    def _plan_t(self, pl):
        """The plan as the CPU uint8 tensor the torch ops take (cached per plan object)."""
        t = self._plan_tensors.get(id(pl))
        if t is None or t[0] is not pl:
            t = (pl, torch.frombuffer(bytearray(bytes(pl)), dtype=torch.uint8))
            self._plan_tensors[id(pl)] = t
        return t[1]

    def _op_batch(self, X, Y, batch_size, mode, idx, perm_seed, full_bayes=False):
        X, Y = self._prep_batch(X, Y, stage=mode == N.BATCH_DIRECT)
        B = X.shape[0] if mode == N.BATCH_DIRECT else int(batch_size)
        pl, ws = self.plan_ws(B, full_bayes=full_bayes)
        if idx is not None:
            idx = torch.as_tensor(idx).to(device=self.dev, dtype=torch.int32).contiguous()
        iters = X.shape[0] // B if mode == N.BATCH_EPOCH else 0
        return pl, ws, X, Y, idx, iters, _i64(perm_seed)

    def step(self, X, Y, data_size, lr, beta, T, resample=False, xi=None, xi_resample=None,
             build=True, omega=None, batch_size=None, mode=N.BATCH_DIRECT, idx=None,
             perm_seed=0, full_bayes=False, xi_hyp=None, xi_hyp_resample=None, z=None):
        """One sgmcmc_update (default: X, Y are the batch, DGPRF_BATCH_DIRECT) through the
        dgprf::sghmc_step_ torch op.  full_bayes: also update the trainable hyper-parameters
        (models/dgp.py:199-216); Omega, c and sigma^2 are rebuilt on the device afterwards."""
        if full_bayes:
            self._check_full_bayes()
            self.hyper_epoch += 1  # the device rewrites hyp / Omega: resident projections stale
        pl, ws, X, Y, idx, iters, ps = self._op_batch(X, Y, batch_size, mode, idx, perm_seed,
                                                      full_bayes)
        if build:
            self.build_omega()
        dv = lambda t: None if t is None else as_device(t, self.dev)
        ops().sghmc_step_(
            self._plan_t(pl), self.theta, self.mom, self.omega if omega is None else omega,
            self.der, self.mass, ws, self.step_ctr, _i64(self.seed), X, Y, int(mode), iters, ps,
            idx, float(lr), float(beta), float(T), float(data_size), bool(resample), dv(xi),
            dv(xi_resample), bool(full_bayes), self.z if z is None else z, self.hyp, self.hmom,
            self.hmass, dv(xi_hyp), dv(xi_hyp_resample))
        self._release_stage()

    def grad(self, X, Y, data_size, build=True, omega=None, batch_size=None,
             mode=N.BATCH_DIRECT, idx=None, perm_seed=0, full_bayes=False, z=None):
        """dU/dW for every layer and chain -> [C, w_total] (dgprf::potential_grad); full_bayes:
        w.r.t. every trainable variable -> [C, w_total + hyp_total] (hyp layout after W)."""
        if full_bayes and self.C > 1 and not self.per_chain_hyp:
            raise ValueError("full_bayesian=True with several chains needs per_chain_hyp=True")
        pl, ws, X, Y, idx, iters, ps = self._op_batch(X, Y, batch_size, mode, idx, perm_seed,
                                                      full_bayes)
        if build:
            self.build_omega()
        g = ops().potential_grad(
            self._plan_t(pl), self.theta, self.omega if omega is None else omega, self.der,
            self.mass, ws, self.step_ctr, X, Y, int(mode), iters, ps, idx, float(data_size),
            bool(full_bayes), self.z if z is None else z, self.hyp, self.hmom, self.hmass)
        self._release_stage()
        return g

    def _release_stage(self):
        if self._staged:
            self._staged = False
            self._stage.release()

    def graph(self, X_all, Y_all, batch_size, data_size, lr, beta, T, steps_per_graph,
              schedule=N.SCHED_CONST, start_step=0, cycle_length=1, resample_head=False,
              perm_seed=0, full_bayes=False, fresh_z=0):
        """hipGraph of `steps_per_graph` on-device-minibatched steps (DGPRF_BATCH_EPOCH);
        fresh_z: layers (bit mask) whose z is redrawn every step (random_fixed=False)."""
        if full_bayes:
            self._check_full_bayes()
            self.hyper_epoch += 1  # its replays rewrite hyp / Omega on the device
        # W-only steps of a wide first layer with fixed z gather their rows of the dataset's
        # resident X Omega_1 (graphs hold its pointer; refreshed in place here when stale, so a
        # cached graph's rows follow the current Omega_1)
        a1 = None if (full_bayes or (fresh_z & 1)) else self.dataset_a1(X_all)
        # a graph holds the resident projection's buffer and the Philox key it was captured with
        key = (X_all.data_ptr(), tuple(X_all.shape), Y_all.data_ptr(), tuple(Y_all.shape),
               int(batch_size), float(data_size), float(lr), float(beta), float(T),
               int(steps_per_graph), int(schedule), int(start_step), int(cycle_length),
               bool(resample_head), int(perm_seed), bool(full_bayes), int(fresh_z),
               0 if a1 is None else a1.data_ptr(), int(self.seed))
        if key in self._graphs:
            g = self._graphs.pop(key)  # most recently used last
            self._graphs[key] = g
            return g
        if len(self._graphs) >= self.MAX_GRAPHS:
            # bounded: evict the least recently used.  Replays are asynchronous, so the stream
            # drains before an evicted graph's executable can be destroyed (_Graph.__del__).
            torch.cuda.current_stream(self.dev).synchronize()
            while len(self._graphs) >= self.MAX_GRAPHS:
                self._graphs.pop(next(iter(self._graphs)))
        pl, ws = self.plan_ws(batch_size, fresh_z, full_bayes)
        iters = X_all.shape[0] // int(batch_size)
        ch = self.chain_struct(ws)
        bt = self.batch_struct(X_all, Y_all, N.BATCH_EPOCH, iters=iters, perm_seed=perm_seed)
        if a1 is not None:
            bt.A1 = a1.data_ptr()
        st = self.step_struct(lr, beta, T, data_size, False, schedule, start_step, cycle_length,
                              resample_head, full_bayes=full_bayes)
        h = ctypes.c_void_p()
        N.call("dgprf_graph_create_sghmc", ctypes.byref(h), ctypes.byref(pl), ctypes.byref(ch),
               ctypes.byref(bt), ctypes.byref(st), int(steps_per_graph))
        g = _Graph(h, (X_all, Y_all, ws, a1), int(steps_per_graph),
                   weakref.ref(self) if full_bayes else None)
        self._graphs[key] = g
        return g

    def profile_step(self, X_all, Y_all, batch_size, data_size, lr, beta, T, reps=200,
                     perm_seed=0):
        """Average device ms of the event pair around each step kernel (hipEvents,
        dgprf_profile_step): {'fwd': [L], 'bwd': [L], 'update': float, 'empty': float,
        'agemm': float}, 'empty' being an event pair with no kernel between (the pair's own cost),
        'agemm' the A_1 = X Omega_1 GEMM of a wide first layer (0 without one)."""
        pl, ws, bt, keep = self._batch(X_all, Y_all, batch_size, N.BATCH_EPOCH, None, perm_seed)
        ch = self.chain_struct(ws)
        st = self.step_struct(lr, beta, T, data_size)
        ms = (ctypes.c_float * (2 * self.L + 3))()
        N.call("dgprf_profile_step", ctypes.byref(pl), ctypes.byref(ch), ctypes.byref(bt),
               ctypes.byref(st), int(reps), ctypes.cast(ms, ctypes.c_void_p), stream())
        v = list(ms)
        return {"fwd": v[:self.L], "bwd": v[self.L:2 * self.L], "update": v[2 * self.L],
                "empty": v[2 * self.L + 1], "agemm": v[2 * self.L + 2]}

    # ---------------------------------------------------------------- forward / predictive
    def forward(self, X, Y=None, f_out=False, logp=False, se=False, lse=None, omega=None,
                build=True):
        """dgprf_forward over all rows of X for every chain.

        Returns a dict with the requested outputs ('F' = list of per-layer [C, n, g_l] when
        f_out='all', or the last layer only when f_out=True; 'logp', 'se' = [C, n]).
        `lse` = (m, s, se_sum) accumulators [C, n] updated in place.
        """
        X = as_device(X, self.dev)
        n = X.shape[0]
        if X.dim() != 2 or X.shape[1] != self.spec.d_in:
            raise ValueError(f"X must be [n, {self.spec.d_in}], got {tuple(X.shape)}")
        if build:
            self.build_omega()
        mask = 0
        if f_out:
            for l in range(self.L):
                if f_out == "all" or l == self.L - 1:
                    mask |= 1 << l
        Yd = None
        if Y is not None:
            Yd = as_device(Y, self.dev)
            if Yd.dim() == 1:
                Yd = Yd[:, None]
        m = s = e = None
        if lse is not None:
            m, s, e = lse
        om = self.omega if omega is None else omega
        Fs, lp, sq = ops().forward(self._plan_t(self.layout), self.theta, om, self.der, X, Yd,
                                   mask, bool(logp), bool(se), m, s, e, self.forward_scratch(n))
        out = {}
        if f_out:
            out["F"] = list(Fs)
        if logp:
            out["logp"] = lp
        if se:
            out["se"] = sq
        return out

    def forward_samples(self, thetas, X, Y, lse, omega=None, build=True, a1=None):
        """Fold S posterior samples of every chain (thetas [S, C, w_total]) into the LSE
        accumulators lse = (m, s, se_sum) [C, n] in sample order (dgprf::forward_samples): two
        samples per pass with layer 0 shared where the model is lean (every layer d, g <= 8);
        a1 = dataset_a1(X) for a wide first layer (no A_1 GEMM per sample)."""
        X = as_device(X, self.dev)
        Yd = as_device(Y, self.dev)
        if Yd.dim() == 1:
            Yd = Yd[:, None]
        thetas = as_device(thetas, self.dev)
        if thetas.dim() == 2:
            thetas = thetas[:, None, :]
        if X.dim() != 2 or X.shape[1] != self.spec.d_in:
            raise ValueError(f"X must be [n, {self.spec.d_in}], got {tuple(X.shape)}")
        if build:
            self.build_omega()
        m, s, e = lse
        om = self.omega if omega is None else omega
        ops().forward_samples(self._plan_t(self.layout), thetas, om, self.der, X, a1, Yd, m, s, e,
                              self.forward_scratch(X.shape[0], thetas.shape[0]))

    def forward_scratch(self, n, n_samples=0):
        """Engine-owned scratch of dgprf_forward for n rows (the wide-first-layer A_1 chunks) or,
        with n_samples, of dgprf_forward_samples (also every sample's per-row log p, so all sample
        pairs run in one launch); grown on demand and reused, so the predictive loop allocates
        nothing per sample."""
        need = ctypes.c_int64(0)
        if n_samples:
            N.call("dgprf_forward_samples_scratch", ctypes.byref(self.layout), int(n),
                   int(n_samples), ctypes.byref(need))
        else:
            N.call("dgprf_forward_scratch", ctypes.byref(self.layout), int(n), ctypes.byref(need))
        if need.value == 0:
            return None
        if self._fwd_scratch is None or self._fwd_scratch.numel() < need.value:
            self._fwd_scratch = torch.empty(need.value, dtype=_F32, device=self.dev)
        return self._fwd_scratch

    def set_forward_path(self, path=N.FWD_AUTO, agemm_chunk_rows=0):
        """Pin the predictive forward path (N.FWD_*) and the A_1 chunk size — parity tests of
        each path; the product default is FWD_AUTO."""
        self.layout.fwd_path = int(path)
        self.layout.agemm_chunk_rows = int(agemm_chunk_rows)
        N.call("dgprf_plan_init", ctypes.byref(self.layout))
        self._plan_tensors.pop(id(self.layout), None)

    def rf_project(self, X, omega, out=None):
        """A = X Omega of one RF layer (layers/rf_layers.py:42, 88) through dgprf_rf_project — the
        hand-written MFMA GEMM of the wide first layer.  X [n, >= d] (row stride X.shape[1]),
        omega [d, R] -> A [n, R]."""
        X = as_device(X, self.dev)
        omega = as_device(omega, self.dev)
        if X.dim() != 2 or omega.dim() != 2:
            raise ValueError("rf_project: X [n, ldx] and omega [d, R] must be 2-D")
        n, ldx = X.shape
        d, R = omega.shape
        if ldx < d:
            raise ValueError(f"rf_project: X has {ldx} columns, omega needs {d}")
        if out is None:
            out = torch.empty(n, R, dtype=_F32, device=self.dev)
        elif (tuple(out.shape) != (n, R) or out.dtype != _F32 or not out.is_contiguous()
              or out.device != X.device):
            raise ValueError(f"rf_project: out must be a contiguous fp32 [{n}, {R}] tensor on "
                             f"{X.device}, got {tuple(out.shape)} {out.dtype} on {out.device}")
        N.call("dgprf_rf_project", ptr(X), int(n), int(ldx), int(d), ptr(omega), int(R), ptr(out),
               stream())
        return out

    def prior_w(self):
        out = torch.empty(self.C, dtype=_F32, device=self.dev)
        N.call("dgprf_prior_w", ctypes.byref(self.layout), ptr(self.theta), ptr(out), stream())
        return out

    # ---------------------------------------------------------------- preconditioner
    def welford(self, grad, mean, m2, k, full_bayes=False):
        N.call("dgprf_welford_update", ctypes.byref(self.layout), ptr(grad), ptr(mean), ptr(m2),
               int(k), int(bool(full_bayes)), stream())

    def mass_estimate(self, mean, m2, K, centered, full_bayes=False):
        """W masses [C, L]; full_bayes: also (hyper masses [C, N.HMASS])."""
        out = torch.empty(self.C, self.L, dtype=_F32, device=self.dev)
        hout = torch.zeros(self.C, N.HMASS, dtype=_F32, device=self.dev) if full_bayes else None
        N.call("dgprf_mass_estimate", ctypes.byref(self.layout), ptr(mean), ptr(m2), int(K),
               int(bool(centered)), int(bool(full_bayes)), ptr(out), ptr(hout), stream())
        return (out, hout) if full_bayes else out

    def hyper_slots(self):
        """The trainable hyper-parameter variables of full_bayesian=True as
        (hmass slot, hyp offset, length) — log_amp, log_inv_ls, mean per layer, then lik_log_var."""
        pl, sp = self.layout, self.spec
        out = []
        for l in range(self.L):
            if sp.hyp_flags & N.HYP_KERNEL:
                out.append((l, l, 1))
                out.append((8 + l, pl.lis_off[l], pl.d[l] if sp.ard[l] else 1))
            if sp.hyp_flags & N.HYP_MEAN:
                out.append((16 + l, pl.mean_off[l], pl.d[l]))
        if (sp.hyp_flags & N.HYP_LIK) and sp.likelihood == N.LIK_GAUSSIAN:
            out.append((24, self.L, 1))
        return out

    def sghmc_update(self, grad, lr, beta, T, data_size, resample=False, xi=None,
                     xi_resample=None):
        """Stand-alone update from a given gradient [C, w_total] (dgprf_sghmc_update)."""
        st = self.step_struct(lr, beta, T, data_size, resample,
                              xi=None if xi is None else as_device(xi, self.dev),
                              xi_resample=None if xi_resample is None else as_device(xi_resample, self.dev))
        grad = as_device(grad, self.dev)
        N.call("dgprf_sghmc_update", ctypes.byref(self.layout), ptr(self.theta), ptr(self.mom),
               ptr(grad), ptr(self.mass), ptr(self.step_ctr), self.seed, ctypes.byref(st),
               stream())


class _Graph:
    def __init__(self, handle, keep, steps=0, hyper_engine=None):
        self.h = handle
        self._keep = keep
        self.steps = steps  # SGHMC steps one replay runs
        # full_bayesian=True graphs: every replay rewrites hyp / Omega on the device, which torch's
        # version counters do not see — each launch advances the engine's hyper_epoch, so a
        # resident projection (dataset_a1) made from the old Omega_1 is recomputed
        self._hyper_engine = hyper_engine

    def launch(self):
        if self._hyper_engine is not None:
            eng = self._hyper_engine()
            if eng is not None:
                eng.hyper_epoch += 1
        N.call("dgprf_graph_launch", self.h, stream())

    def __del__(self):
        try:
            if self.h:
                N.lib().dgprf_graph_destroy(self.h)
        except Exception:
            pass


def lse_finalize(lse_m, lse_s, se_sum, s_total, y_std=1.0, lse_out=False):
    """Posterior-predictive LL / RMSE from stacked accumulators [parts, n] (dgprf::lse_finalize):
    returns (float64 [LL, RMSE] on the device, per-point LSE [n] or None)."""
    out, lo = ops().lse_finalize(lse_m.contiguous(), lse_s.contiguous(),
                                 None if se_sum is None else se_sum.contiguous(), float(s_total),
                                 float(y_std), bool(lse_out))
    return out, (lo if lse_out else None)
