"""ctypes binding of libdgprf.so — the C-ABI declared in include/dgprf.h.

The library is built in-tree (``make -C dgp-rf-mcmc_amd/csrc`` or ``__graft_entry__.build()``) and
loaded from this directory.  There is no fallback: if the library or a HIP device is missing,
every compute entry point raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DGPRF_LIB", os.path.join(_HERE, "libdgprf.so"))

MAX_LAYERS = 8
MAX_G = 64
MAX_D = 2048

RBF, ARC = 0, 1
LIK_GAUSSIAN, LIK_SOFTMAX = 0, 1
BATCH_DIRECT, BATCH_INDEXED, BATCH_EPOCH = 0, 1, 2
SCHED_CONST, SCHED_CYCLICAL = 0, 1
RNG_NOISE, RNG_RESAMPLE, RNG_Z, RNG_W, RNG_MOMENTS = 1, 2, 3, 4, 5
RNG_HYPER, RNG_HYPER_RESAMPLE = 6, 7
HYP_KERNEL, HYP_LIK, HYP_MEAN = 1, 2, 4
HMASS = 32  # hmass slots: log_amp l -> l, log_inv_ls l -> 8 + l, mean l -> 16 + l, lik_log_var -> 24
ABI_VERSION = 10
FWD_AUTO, FWD_ROWS, FWD_NO_AGEMM, FWD_TILE, FWD_ROWS16, FWD_ROWS8 = 0, 1, 2, 3, 4, 5

E_ARG, E_SHAPE, E_HIP, E_PLAN = -1, -2, -3, -4

_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_u64 = ctypes.c_uint64
_fp = ctypes.POINTER(ctypes.c_float)
_vp = ctypes.c_void_p
_L = MAX_LAYERS


class Plan(ctypes.Structure):
    """dgprf_plan_t."""
    _fields_ = [
        ("n_layers", _i32), ("d_in", _i32), ("d_out", _i32), ("input_cat", _i32),
        ("likelihood", _i32), ("batch", _i32), ("n_chains", _i32),
        ("kind", _i32 * _L), ("n_rf", _i32 * _L), ("n_gp", _i32 * _L),
        ("hyp_flags", _i32), ("hyp_per_chain", _i32), ("ard", _i32 * _L),
        ("fwd_path", _i32), ("agemm_chunk_rows", _i32), ("fresh_z", _i32), ("bwd_tiles", _i32),
        ("initialised", _i32),
        ("d", _i32 * _L), ("P", _i32 * _L), ("ns", _i32 * _L), ("cpw", _i32 * _L),
        ("n_row_tiles", _i32), ("n_rt_pad", _i32), ("rt_per_group", _i32), ("n_gw_rows", _i32),
        ("rg_full_bayes", _i32), ("fold_out", _i32),
        ("omega_off", _i64 * _L), ("w_off", _i64 * _L), ("lis_off", _i64 * _L),
        ("mean_off", _i64 * _L), ("fp_off", _i64 * _L), ("dxp_off", _i64 * _L),
        ("gwp_off", _i64), ("logp_off", _i64),
        ("omega_total", _i64), ("w_total", _i64), ("hyp_total", _i64), ("der_total", _i64),
        ("ws_chain", _i64), ("ws_total", _i64), ("hpp_off", _i64 * _L), ("hpl_off", _i64),
        ("xb_off", _i64), ("yb_off", _i64),
        ("yb_cols", _i32), ("pad0", _i32), ("a0_off", _i64), ("omf_off", _i64),
    ]


class Chain(ctypes.Structure):
    """dgprf_chain_t."""
    _fields_ = [("theta", _vp), ("mom", _vp), ("omega", _vp), ("der", _vp), ("mass", _vp),
                ("z", _vp), ("hyp", _vp), ("hmom", _vp), ("hmass", _vp),
                ("ws", _vp), ("step", _vp), ("seed", _u64)]


class Batch(ctypes.Structure):
    """dgprf_batch_t."""
    _fields_ = [("X", _vp), ("Y", _vp), ("idx", _vp), ("n_data", _i64), ("y_cols", _i32),
                ("mode", _i32), ("iters_per_epoch", _i64), ("perm_seed", _u64), ("A1", _vp)]


class Step(ctypes.Structure):
    """dgprf_step_t."""
    _fields_ = [("lr", ctypes.c_float), ("momentum_decay", ctypes.c_float),
                ("temperature", ctypes.c_float), ("data_size", ctypes.c_float),
                ("resample_moments", _i32), ("schedule", _i32), ("step_offset", _i32),
                ("grad_only", _i32), ("start_step", _i64), ("cycle_length", _i64),
                ("resample_in_cycle_head", _i32), ("full_bayes", _i32), ("xi", _vp),
                ("xi_resample", _vp), ("xi_hyp", _vp), ("xi_hyp_resample", _vp)]


# name -> (restype, argtypes); must match include/dgprf.h exactly.
SIGNATURES = {
    "dgprf_abi_version": (_i32, []),
    "dgprf_error_string": (ctypes.c_char_p, [_i32]),
    "dgprf_plan_init": (_i32, [ctypes.POINTER(Plan)]),
    "dgprf_philox_normal": (_i32, [_vp, _i64, _u64, _u64, ctypes.c_uint32, _vp]),
    "dgprf_omega_build": (_i32, [ctypes.POINTER(Plan), _vp, _vp, _vp, _vp, _vp]),
    "dgprf_sghmc_step": (_i32, [ctypes.POINTER(Plan), ctypes.POINTER(Chain),
                                ctypes.POINTER(Batch), ctypes.POINTER(Step), _vp]),
    "dgprf_potential_grad": (_i32, [ctypes.POINTER(Plan), ctypes.POINTER(Chain),
                                    ctypes.POINTER(Batch), ctypes.c_float, _i32, _vp, _vp]),
    "dgprf_graph_create_sghmc": (_i32, [ctypes.POINTER(_vp), ctypes.POINTER(Plan),
                                        ctypes.POINTER(Chain), ctypes.POINTER(Batch),
                                        ctypes.POINTER(Step), _i32]),
    "dgprf_graph_launch": (_i32, [_vp, _vp]),
    "dgprf_graph_destroy": (_i32, [_vp]),
    "dgprf_forward_samples": (_i32, [ctypes.POINTER(Plan), _vp, _i32, _vp, _vp, _vp, _vp, _vp, _i32,
                                     _i64, _vp, _vp, _vp, _vp, _i64, _vp]),
    "dgprf_profile_step": (_i32, [ctypes.POINTER(Plan), ctypes.POINTER(Chain),
                                  ctypes.POINTER(Batch), ctypes.POINTER(Step), _i32, _vp, _vp]),
    "dgprf_forward_scratch": (_i32, [ctypes.POINTER(Plan), _i64, ctypes.POINTER(_i64)]),
    "dgprf_forward_samples_scratch": (_i32, [ctypes.POINTER(Plan), _i64, _i32,
                                             ctypes.POINTER(_i64)]),
    "dgprf_forward": (_i32, [ctypes.POINTER(Plan), _vp, _vp, _vp, _vp, _vp, _i32, _i64,
                             ctypes.POINTER(_vp), _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp]),
    "dgprf_lse_finalize": (_i32, [_vp, _vp, _vp, _i32, _i64, ctypes.c_double, ctypes.c_float,
                                  ctypes.c_float, _vp, _vp, _vp]),
    "dgprf_rf_omega": (_i32, [_i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "dgprf_rf_features": (_i32, [_i32, _vp, _i64, _i32, _vp, _i32, _vp, _vp, _vp]),
    "dgprf_gp_matmul": (_i32, [_vp, _i64, _i32, _vp, _i32, _vp, _vp]),
    "dgprf_rf_project": (_i32, [_vp, _i64, _i32, _i32, _vp, _i32, _vp, _vp]),
    "dgprf_prior_w": (_i32, [ctypes.POINTER(Plan), _vp, _vp, _vp]),
    "dgprf_sghmc_update": (_i32, [ctypes.POINTER(Plan), _vp, _vp, _vp, _vp, _vp, _u64,
                                  ctypes.POINTER(Step), _vp]),
    "dgprf_welford_update": (_i32, [ctypes.POINTER(Plan), _vp, _vp, _vp, _i32, _i32, _vp]),
    "dgprf_mass_estimate": (_i32, [ctypes.POINTER(Plan), _vp, _vp, _i32, _i32, _i32, _vp, _vp,
                                   _vp]),
}

_lib = None


class DgprfError(RuntimeError):
    """A libdgprf entry point returned an error code."""

    def __init__(self, fn, code):
        msg = _lib.dgprf_error_string(code).decode() if _lib is not None else str(code)
        super().__init__(f"{fn} failed: {msg} (code {code})")
        self.code = code


def lib():
    """Load libdgprf.so (once).  Raises ImportError if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libdgprf.so not found at {LIB_PATH}: build it with "
            "`make -C dgp-rf-mcmc_amd/csrc` (hipcc --offload-arch=gfx950). "
            "There is no CPU fallback.")
    h = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        f = getattr(h, name)
        f.restype = res
        f.argtypes = args
    if h.dgprf_abi_version() != ABI_VERSION:
        raise ImportError("libdgprf.so ABI version mismatch")
    _lib = h
    return h


# next to the C-ABI library it links ($ORIGIN), so a DGPRF_LIB build directory carries its own pair
TORCH_LIB_PATH = os.path.join(os.path.dirname(LIB_PATH), "libdgprf_torch.so")
_ops = None


def torch_ops():
    """Register the dgprf torch operators (libdgprf_torch.so: TORCH_LIBRARY(dgprf, m) over this
    C-ABI) once and return torch.ops.dgprf.  Raises ImportError if it has not been built."""
    global _ops
    if _ops is None:
        import torch
        lib()  # libdgprf.so first (the op library links it)
        if not os.path.exists(TORCH_LIB_PATH):
            raise ImportError(f"libdgprf_torch.so not found at {TORCH_LIB_PATH}: build it with "
                              "`make -C dgp-rf-mcmc_amd/csrc`. There is no CPU fallback.")
        torch.ops.load_library(TORCH_LIB_PATH)
        _ops = torch.ops.dgprf
    return _ops


def call(name, *args):
    """Call an entry point and raise DgprfError on a non-zero return code."""
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        if rc == E_SHAPE:
            raise ValueError(f"{name}: unsupported shape ({lib().dgprf_error_string(rc).decode()})")
        raise DgprfError(name, rc)
    return rc


def make_plan(d_in, d_out, kinds, n_rf, n_gp, input_cat, likelihood, batch, n_chains,
              hyp_flags=0, hyp_per_chain=0, ard=None):
    """Fill and derive a Plan (dgprf_plan_init is host-only: usable without a GPU).
    hyp_flags: HYP_* groups trainable under full_bayesian=True; ard[l]: per-dimension length
    scales (the DGP_RF default, models/dgp.py:80-85) or one scalar."""
    L = len(kinds)
    if not 1 <= L <= MAX_LAYERS:
        raise ValueError(f"n_hidden_layers must be in [1, {MAX_LAYERS}]")
    p = Plan()
    p.n_layers, p.d_in, p.d_out = L, int(d_in), int(d_out)
    p.input_cat, p.likelihood = int(bool(input_cat)), int(likelihood)
    p.batch, p.n_chains = int(batch), int(n_chains)
    p.hyp_flags, p.hyp_per_chain = int(hyp_flags), int(bool(hyp_per_chain))
    for l in range(L):
        p.kind[l], p.n_rf[l], p.n_gp[l] = int(kinds[l]), int(n_rf[l]), int(n_gp[l])
        p.ard[l] = 1 if ard is None else int(bool(ard[l]))
    call("dgprf_plan_init", ctypes.byref(p))
    return p
