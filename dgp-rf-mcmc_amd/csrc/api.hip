// api.hip — extern "C" entry points of libdgprf.so (declared in include/dgprf.h).
//
// Host-side validation and planning mirror the reference's constructor and assertions
// (models/dgp.py:34-52, 74-115; kernels/RBF.py:19-27; kernels/arc_cosine.py:13-16): configuration
// errors are reported as return codes before anything is enqueued.
#include <cstdlib>
#include <cstring>
#include <new>

#include "dgprf_internal.h"
#include "step_common.h"

namespace {

inline int64_t align4(int64_t x) { return (x + 3) & ~int64_t(3); }

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

int hip_rc(hipError_t e) { return e == hipSuccess ? DGPRF_OK : DGPRF_E_HIP; }

StepDev make_step_dev(const dgprf_plan_t& pl, const dgprf_chain_t& ch, const dgprf_batch_t& b,
                      int32_t step_offset) {
  StepDev sd;
  sd.theta = ch.theta;
  sd.mom = ch.mom;
  sd.omega = ch.omega;
  sd.der = ch.der;
  sd.mass = ch.mass;
  sd.ws = ch.ws;
  sd.step = ch.step;
  sd.grad_out = nullptr;
  sd.seed = ch.seed;
  sd.bd.X = b.X;
  sd.bd.Y = b.Y;
  sd.bd.idx = b.idx;
  sd.bd.n_data = b.n_data;
  sd.bd.iters = b.iters_per_epoch;
  sd.bd.perm_seed = b.perm_seed;
  sd.bd.y_cols = b.y_cols;
  sd.bd.mode = b.mode;
  // resident A_1 rows (wide first layer, fixed Omega_1, a dataset to gather from); enqueue_step
  // drops it for full-Bayes steps (Omega_1 changes in-step).  Per-chain hyper-parameters with
  // several chains give every chain its own Omega_1, which one [n][R_1] projection cannot serve:
  // ignored there (the GEMM runs per chain)
  const bool res = b.A1 && pl.a0_off >= 0 && b.mode != DGPRF_BATCH_DIRECT && !(pl.fresh_z & 1) &&
                   pl.n_rf[0] % 4 == 0 && !(pl.hyp_per_chain && pl.n_chains > 1);
  sd.bd.A1 = res ? b.A1 : nullptr;
  sd.bd.a1_ld = pl.n_rf[0];
  sd.bd.pad = 0;
  sd.step_offset = step_offset;
  sd.full_bayes = 0;
  const bool pc = pl.hyp_per_chain != 0;
  sd.om_cs = pc ? pl.omega_total : 0;
  sd.der_cs = pc ? pl.der_total : 0;
  sd.hyp_cs = pc ? pl.hyp_total : 0;
  sd.z = ch.z;
  sd.hyp = ch.hyp;
  sd.hmom = ch.hmom;
  sd.hmass = ch.hmass;
  return sd;
}

UpdateDev make_update_dev(const dgprf_step_t& st) {
  UpdateDev ud;
  ud.lr = st.lr;
  ud.beta = st.momentum_decay;
  ud.temperature = st.temperature;
  ud.data_size = st.data_size;
  ud.resample = st.resample_moments;
  ud.schedule = st.schedule;
  ud.grad_only = st.grad_only;
  ud.resample_head = st.resample_in_cycle_head;
  ud.start_step = st.start_step;
  ud.cycle_length = st.cycle_length > 0 ? st.cycle_length : 1;
  ud.xi = st.xi;
  ud.xi_resample = st.xi_resample;
  ud.xi_hyp = st.xi_hyp;
  ud.xi_hyp_resample = st.xi_hyp_resample;
  return ud;
}

int check_plan(const dgprf_plan_t* pl) {
  if (!pl) return DGPRF_E_ARG;
  if (pl->initialised != 1) return DGPRF_E_PLAN;
  return DGPRF_OK;
}

int check_chain(const dgprf_chain_t* ch) {
  if (!ch || !ch->theta || !ch->mom || !ch->omega || !ch->der || !ch->mass || !ch->ws || !ch->step)
    return DGPRF_E_ARG;
  return DGPRF_OK;
}

int check_batch(const dgprf_plan_t& pl, const dgprf_batch_t* b) {
  if (!b || !b->X || !b->Y || b->y_cols < 1) return DGPRF_E_ARG;
  if (b->mode == DGPRF_BATCH_DIRECT) {
    if (b->n_data < pl.batch) return DGPRF_E_SHAPE;
  } else if (b->mode == DGPRF_BATCH_INDEXED) {
    if (!b->idx) return DGPRF_E_ARG;
  } else if (b->mode == DGPRF_BATCH_EPOCH) {
    if (b->iters_per_epoch < 1 || b->iters_per_epoch * (int64_t)pl.batch > b->n_data ||
        b->n_data > (int64_t)0xFFFFFFFFll)
      return DGPRF_E_SHAPE;
  } else {
    return DGPRF_E_ARG;
  }
  if (pl.likelihood == DGPRF_LIK_GAUSSIAN && b->y_cols < pl.n_gp[pl.n_layers - 1]) return DGPRF_E_SHAPE;
  return DGPRF_OK;
}

int check_step(const dgprf_step_t* st) {
  if (!st) return DGPRF_E_ARG;
  if (!(st->data_size > 0.f)) return DGPRF_E_ARG;
  if (st->schedule != DGPRF_SCHED_CONST && st->schedule != DGPRF_SCHED_CYCLICAL) return DGPRF_E_ARG;
  return DGPRF_OK;
}

// [gather rows] fwd for every layer, bwd in reverse, then the update.  prep_gather: gather this
// step's minibatch rows first; gather_next: the update kernel gathers step t+1's rows (graph
// replays, where the next step is known to follow).  The update kernel sums the gW partials and
// updates every W (and the full-Bayes hyper-parameters).
hipError_t enqueue_step(const dgprf_plan_t& pl, const StepDev& sd_in, const UpdateDev& ud,
                        hipStream_t s, bool prep_gather = true, bool gather_next = false,
                        bool advance = false) {
  hipError_t e = hipSuccess;
  StepDev sd = sd_in;
  if (sd.full_bayes) sd.bd.A1 = nullptr;  // Omega_1 changes every full-Bayes step: the GEMM
  if (prep_gather) e = dgprf::launch_gather(pl, sd, s);
  // random_fixed=False layers: this step's Omega from fresh z (layers/rf_layers.py:39-41)
  if (e == hipSuccess && pl.fresh_z) e = dgprf::launch_fresh_omega(pl, sd, s);
  if (dgprf_sk::step_fused_fwd(pl)) {  // large B, one chain: one all-layer forward launch
    if (e == hipSuccess) e = dgprf::launch_step_fwd_fused(pl, sd, s);
  } else {
    // a folded output layer (plan.fold_out, W-only) is formed inside its backward: no launch
    const int nf = pl.fold_out && !sd.full_bayes ? pl.n_layers - 1 : pl.n_layers;
    for (int l = 0; l < nf && e == hipSuccess; ++l) e = dgprf::launch_step_fwd(pl, sd, l, s);
  }
  for (int l = pl.n_layers - 1; l >= 0 && e == hipSuccess; --l)
    e = dgprf::launch_step_bwd(pl, sd, l, s);
  if (e == hipSuccess) e = dgprf::launch_step_update(pl, sd, ud, nullptr, s, gather_next, advance);
  return e;
}

// full_bayesian=True needs the hyper-parameter state, and per-chain hyper-parameters when several
// chains step at once
int check_full_bayes(const dgprf_plan_t& pl, const dgprf_chain_t& ch) {
  if (!ch.z || !ch.hyp || !ch.hmom || !ch.hmass) return DGPRF_E_ARG;
  if (pl.n_chains > 1 && !pl.hyp_per_chain) return DGPRF_E_ARG;
  if (pl.rt_per_group > 1 && !pl.rg_full_bayes) return DGPRF_E_SHAPE;
  return DGPRF_OK;
}

}  // namespace

struct dgprf_graph {
  hipGraph_t graph;
  hipGraphExec_t exec;
};

extern "C" {

int dgprf_abi_version(void) { return DGPRF_ABI_VERSION; }

const char* dgprf_error_string(int code) {
  switch (code) {
    case DGPRF_OK: return "ok";
    case DGPRF_E_ARG: return "invalid argument (null pointer or bad scalar)";
    case DGPRF_E_SHAPE: return "unsupported shape";
    case DGPRF_E_HIP: return "HIP runtime error";
    case DGPRF_E_PLAN: return "plan not initialised (call dgprf_plan_init)";
    default: return "unknown error";
  }
}

int dgprf_plan_init(dgprf_plan_t* pl) {
  if (!pl) return DGPRF_E_ARG;
  pl->initialised = 0;
  const int L = pl->n_layers;
  if (L < 1 || L > DGPRF_MAX_LAYERS) return DGPRF_E_SHAPE;
  if (pl->d_in < 1 || pl->d_out < 1 || pl->batch < 1 || pl->n_chains < 1) return DGPRF_E_SHAPE;
  if (pl->likelihood != DGPRF_LIK_GAUSSIAN && pl->likelihood != DGPRF_LIK_SOFTMAX) return DGPRF_E_ARG;
  if (pl->fwd_path < DGPRF_FWD_AUTO || pl->fwd_path > DGPRF_FWD_ROWS8 || pl->agemm_chunk_rows < 0 ||
      pl->fresh_z < 0 || (pl->fresh_z >> L) != 0 || (pl->bwd_tiles != 0 && pl->bwd_tiles != 1))
    return DGPRF_E_ARG;
  for (int l = 0; l < L; ++l) {
    if (pl->kind[l] != DGPRF_RBF && pl->kind[l] != DGPRF_ARC) return DGPRF_E_ARG;
    if (pl->n_rf[l] < 1 || pl->n_gp[l] < 1 || pl->n_gp[l] > DGPRF_MAX_G) return DGPRF_E_SHAPE;
  }
  if ((pl->hyp_flags & ~(DGPRF_HYP_KERNEL | DGPRF_HYP_LIK | DGPRF_HYP_MEAN)) != 0 ||
      (pl->hyp_per_chain != 0 && pl->hyp_per_chain != 1))
    return DGPRF_E_ARG;
  for (int l = 0; l < L; ++l)
    if (pl->ard[l] != 0 && pl->ard[l] != 1) return DGPRF_E_ARG;
  for (int l = L; l < DGPRF_MAX_LAYERS; ++l) {
    pl->kind[l] = 0;
    pl->n_rf[l] = 0;
    pl->n_gp[l] = 0;
    pl->ard[l] = 0;
  }
  // widths: [d_in, n_gp[:-1]] (+ d_in when input_cat)   models/dgp.py:76-79
  int64_t om = 0, w = 0, lis = 0;
  for (int l = 0; l < DGPRF_MAX_LAYERS; ++l) {
    pl->d[l] = pl->P[l] = pl->ns[l] = pl->cpw[l] = 0;
    pl->omega_off[l] = pl->w_off[l] = pl->lis_off[l] = pl->mean_off[l] = 0;
    pl->fp_off[l] = pl->dxp_off[l] = pl->hpp_off[l] = 0;
  }
  for (int l = 0; l < L; ++l) {
    pl->d[l] = l == 0 ? pl->d_in : pl->n_gp[l - 1] + (pl->input_cat ? pl->d_in : 0);
    if (pl->d[l] > DGPRF_MAX_D) return DGPRF_E_SHAPE;
    pl->P[l] = pl->kind[l] == DGPRF_RBF ? 2 * pl->n_rf[l] : pl->n_rf[l];  // models/dgp.py:103,107
    pl->omega_off[l] = om;
    om = align4(om + (int64_t)pl->d[l] * pl->n_rf[l]);
    pl->w_off[l] = w;
    w = align4(w + (int64_t)pl->P[l] * pl->n_gp[l]);
    // step decomposition: <= 16 feature slices of 4 waves x cpw 16-feature chunks.  Several
    // chains per launch fill the chip with chains, and wider slices then cut the per-slice partial
    // round trips: >= 4 chunks per wave from 4 chains, >= 8 from 16 when g_l <= 16 (config 2,
    // chain-steps/s at 4 / 8 / 16 / 64 chains: 91.6k / 118k / 144k / 170k with 16 slices, 103k /
    // 156k / 209k / 276k with 4, 82k / 150k / 217k / 280k with 2; 2 chains: 16 slices best.
    // Config 3 at 4 / 16 / 64 chains 65k / 94k / 109k -> 87k / 141k / 169k.  Config 4's g = 30
    // layers at 8 chunks per wave: 14.0k -> 11.8k (their whole-slice W / Omega image no longer
    // fits the LDS), hence the g_l bound)
    const int chunks = (pl->n_rf[l] + 15) / 16;
    int cpw = (chunks + 4 * 16 - 1) / (4 * 16);
    const int cmin = pl->n_chains >= 16 && pl->n_gp[l] <= 16 ? 8 : (pl->n_chains >= 4 ? 4 : 1);
    cpw = std::max(cpw, std::min(cmin, (chunks + 3) / 4));
    pl->cpw[l] = cpw < 1 ? 1 : cpw;
    pl->ns[l] = (chunks + 4 * pl->cpw[l] - 1) / (4 * pl->cpw[l]);
  }
  pl->omega_total = om;
  pl->w_total = w;
  // hyp: log_amp[L] | lik_log_var | pad to 4 | log_inv_ls (sum d) | mean (sum d)
  lis = align4(L + 1);
  for (int l = 0; l < L; ++l) {
    pl->lis_off[l] = lis;
    lis += pl->d[l];
  }
  lis = align4(lis);
  for (int l = 0; l < L; ++l) {
    pl->mean_off[l] = lis;
    lis += pl->d[l];
  }
  pl->hyp_total = align4(lis);
  pl->der_total = DGPRF_MAX_LAYERS + 4;
  // workspace (per chain)
  const int B = pl->batch;
  pl->n_row_tiles = (B + 15) / 16;
  int64_t ws = 0;
  // partial buffers always hold DGPRF_NS_MAX slices / a multiple of 16 row tiles; the unused
  // ones stay zero (caller zero-fills the workspace once) so consumers sum a fixed, unrolled
  // count of independent loads in a fixed order.
  for (int l = 0; l < L; ++l) {
    pl->fp_off[l] = ws;
    ws = align4(ws + (int64_t)DGPRF_NS_MAX * B * pl->n_gp[l]);
  }
  for (int l = 1; l < L; ++l) {
    pl->dxp_off[l] = ws;
    ws = align4(ws + (int64_t)DGPRF_NS_MAX * B * pl->n_gp[l - 1]);
  }
  // backward row groups: beyond 16 row tiles every workgroup walks ceil(n_rt / 16) row tiles and
  // keeps its gW in accumulators (k_step_bwd_rg), so the gW partials stay <= 16 rows
  pl->rt_per_group = 1;
  pl->rg_full_bayes = 0;
  pl->fold_out = 0;
  // Many chains per launch (the chip full of chains: throughput, not latency): one row group per
  // chain, so each chain writes ONE gW partial row per parameter instead of one per row tile and the
  // update kernel reads one (at 64 chains it streams 13 rows per parameter of every chain).  Only
  // for wide layers (>= 8 slices each): the row tiles of a chain then run in one workgroup per
  // slice, which a narrow model cannot afford.  B = 200 chain-steps/s at 16 / 64 chains, per-row-
  // tile -> row group: config 4 14.6k / 14.7k -> 17.8k / 19.8k, config 5 15.2k / 15.3k -> 17.8k /
  // 18.0k; config 2 (2 slices) 217k / 280k -> 56k / 179k, config 3 (4) 141k / 168k -> 58k / 159k
  int min_ns = DGPRF_NS_MAX;
  for (int l = 0; l < L; ++l) min_ns = std::min(min_ns, pl->ns[l]);
  const bool mc_rg = pl->n_chains >= DGPRF_MC_RG_CHAINS && pl->n_row_tiles > 1 && min_ns >= 8;
  if ((pl->n_row_tiles > 16 || mc_rg) && !pl->bwd_tiles) {
    bool ok = true, ok_fb = true;
    dgprf_sk::RgCfg c;
    for (int l = 0; l < L; ++l) {
      ok = ok && dgprf_sk::rg_config(*pl, l, false, c);
      ok_fb = ok_fb && dgprf_sk::rg_config(*pl, l, true, c);
    }
    if (ok) {
      pl->rt_per_group = pl->n_row_tiles > 16 ? (pl->n_row_tiles + 15) / 16 : pl->n_row_tiles;
      pl->rg_full_bayes = ok_fb ? 1 : 0;
    }
  }
  pl->n_gw_rows = (pl->n_row_tiles + pl->rt_per_group - 1) / pl->rt_per_group;
  pl->n_rt_pad = (pl->n_gw_rows + 15) / 16 * 16;
  // the update kernel addresses the gW partials with 32-bit buffer offsets
  const int64_t gw_ld = dgprf_sk::gw_row_stride(pl->w_total);
  if ((int64_t)pl->n_rt_pad * gw_ld >= ((int64_t)1 << 29)) return DGPRF_E_SHAPE;
  pl->gwp_off = ws;
  ws = align4(ws + (int64_t)pl->n_rt_pad * gw_ld);
  pl->logp_off = ws;
  ws = align4(ws + B);
  // full-Bayes partials of each backward workgroup: per input dim sum_b X (dA z^T), sum_b X
  // rowsum(dA), then sum dPhi * Phi; and the lik_log_var term per row tile
  for (int l = 0; l < L; ++l) {
    pl->hpp_off[l] = ws;
    ws = align4(ws + (int64_t)pl->n_rt_pad * DGPRF_NS_MAX * align4(2 * pl->d[l] + 1));
  }
  // then DGPRF_MAX_LAYERS uint32 arrival counters of the hyper workgroups and the eager steps'
  // step-advance counter (dgprf_sghmc_step)
  pl->hpl_off = ws;
  ws = align4(ws + pl->n_rt_pad + DGPRF_MAX_LAYERS + 1);
  pl->yb_cols = pl->likelihood == DGPRF_LIK_SOFTMAX ? 1 : pl->n_gp[L - 1];
  pl->xb_off = ws;
  ws = align4(ws + (int64_t)B * pl->d_in);
  pl->yb_off = ws;
  ws = align4(ws + (int64_t)B * pl->yb_cols);
  pl->omf_off = -1;
  if (pl->fresh_z) {
    pl->omf_off = ws;
    ws = align4(ws + om);
  }
  // wide first layer: A_1 = X Omega_1 is one tiled GEMM per step instead of a d-long dependent
  // k-step loop inside every forward / backward chunk; two [align32(B)][R] slabs (its K parts)
  pl->a0_off = -1;
  if (pl->d[0] > 32) {
    pl->a0_off = ws;
    ws = align4(ws + 2 * (int64_t)((B + 31) / 32 * 32) * pl->n_rf[0]);
  }
  // the row-group / row-wave backward kernels address a chain's workspace with 32-bit buffer
  // offsets: refuse the plan here rather than failing every step at launch
  if (pl->rt_per_group > 1 && ws >= ((int64_t)1 << 29)) return DGPRF_E_SHAPE;
  pl->ws_chain = ws;
  pl->ws_total = ws * pl->n_chains;
  pl->fold_out = dgprf_sk::step_fold_out(*pl) ? 1 : 0;
  pl->initialised = 1;
  return DGPRF_OK;
}

int dgprf_philox_normal(float* out, int64_t n, uint64_t seed, uint64_t subsequence,
                        uint32_t purpose, void* stream) {
  if (n < 0 || (n > 0 && !out) || purpose > 255) return DGPRF_E_ARG;
  return hip_rc(dgprf::launch_philox_normal(out, n, seed, subsequence, purpose, as_stream(stream)));
}

int dgprf_omega_build(const dgprf_plan_t* plan, const float* z, const float* hyp, float* omega,
                      float* der, void* stream) {
  int rc = check_plan(plan);
  if (rc) return rc;
  if (!z || !hyp || !omega || !der) return DGPRF_E_ARG;
  return hip_rc(dgprf::launch_omega_build(*plan, z, hyp, omega, der, as_stream(stream)));
}

int dgprf_sghmc_step(const dgprf_plan_t* plan, const dgprf_chain_t* chain,
                     const dgprf_batch_t* batch, const dgprf_step_t* step, void* stream) {
  int rc = check_plan(plan);
  if (!rc) rc = check_chain(chain);
  if (!rc) rc = check_batch(*plan, batch);
  if (!rc) rc = check_step(step);
  if (rc) return rc;
  if (step->full_bayes && (rc = check_full_bayes(*plan, *chain))) return rc;
  if (step->full_bayes && plan->fresh_z) return DGPRF_E_ARG;
  dgprf_step_t st = *step;
  st.grad_only = 0;
  StepDev sd = make_step_dev(*plan, *chain, *batch, st.step_offset);
  sd.full_bayes = st.full_bayes != 0;
  const UpdateDev ud = make_update_dev(st);
  // the update kernel's last workgroup advances the step counter (one launch fewer per call)
  return hip_rc(enqueue_step(*plan, sd, ud, as_stream(stream), true, false, true));
}

int dgprf_potential_grad(const dgprf_plan_t* plan, const dgprf_chain_t* chain,
                         const dgprf_batch_t* batch, float data_size, int32_t full_bayes,
                         float* grad_out, void* stream) {
  int rc = check_plan(plan);
  if (!rc) rc = check_chain(chain);
  if (!rc) rc = check_batch(*plan, batch);
  if (rc) return rc;
  if (!grad_out || !(data_size > 0.f)) return DGPRF_E_ARG;
  if (full_bayes && (rc = check_full_bayes(*plan, *chain))) return rc;
  if (full_bayes && plan->fresh_z) return DGPRF_E_ARG;
  StepDev sd = make_step_dev(*plan, *chain, *batch, 0);
  sd.grad_out = grad_out;
  sd.full_bayes = full_bayes != 0;
  dgprf_step_t st;
  std::memset(&st, 0, sizeof(st));
  st.data_size = data_size;
  st.grad_only = 1;
  return hip_rc(enqueue_step(*plan, sd, make_update_dev(st), as_stream(stream)));
}

int dgprf_graph_create_sghmc(dgprf_graph_handle* out, const dgprf_plan_t* plan,
                             const dgprf_chain_t* chain, const dgprf_batch_t* batch,
                             const dgprf_step_t* step, int32_t steps_per_graph) {
  if (!out) return DGPRF_E_ARG;
  *out = nullptr;
  int rc = check_plan(plan);
  if (!rc) rc = check_chain(chain);
  if (!rc) rc = check_batch(*plan, batch);
  if (!rc) rc = check_step(step);
  if (rc) return rc;
  if (steps_per_graph < 1 || step->xi || step->xi_resample || step->xi_hyp ||
      step->xi_hyp_resample)
    return DGPRF_E_ARG;
  if (step->full_bayes && (rc = check_full_bayes(*plan, *chain))) return rc;
  if (step->full_bayes && plan->fresh_z) return DGPRF_E_ARG;
  hipStream_t cs;
  if (hipStreamCreateWithFlags(&cs, hipStreamNonBlocking) != hipSuccess) return DGPRF_E_HIP;
  hipError_t e = hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal);
  dgprf_step_t st = *step;
  st.grad_only = 0;
  const UpdateDev ud = make_update_dev(st);
  for (int k = 0; k < steps_per_graph && e == hipSuccess; ++k) {
    StepDev sd = make_step_dev(*plan, *chain, *batch, st.step_offset + k);
    sd.full_bayes = st.full_bayes != 0;
    e = enqueue_step(*plan, sd, ud, cs, k == 0, k + 1 < steps_per_graph);
  }
  if (e == hipSuccess) e = dgprf::launch_advance(chain->step, steps_per_graph, cs);
  hipGraph_t g = nullptr;
  const hipError_t e2 = hipStreamEndCapture(cs, &g);
  if (e == hipSuccess) e = e2;
  hipGraphExec_t ex = nullptr;
  if (e == hipSuccess) e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
  (void)hipStreamDestroy(cs);
  if (e != hipSuccess) {
    if (g) (void)hipGraphDestroy(g);
    return DGPRF_E_HIP;
  }
  dgprf_graph* h = new (std::nothrow) dgprf_graph;
  if (!h) {
    (void)hipGraphExecDestroy(ex);
    (void)hipGraphDestroy(g);
    return DGPRF_E_HIP;
  }
  h->graph = g;
  h->exec = ex;
  *out = h;
  return DGPRF_OK;
}

int dgprf_graph_launch(dgprf_graph_handle graph, void* stream) {
  if (!graph) return DGPRF_E_ARG;
  return hip_rc(hipGraphLaunch(graph->exec, as_stream(stream)));
}

int dgprf_graph_destroy(dgprf_graph_handle graph) {
  if (!graph) return DGPRF_OK;
  hipError_t e = hipGraphExecDestroy(graph->exec);
  const hipError_t e2 = hipGraphDestroy(graph->graph);
  delete graph;
  return hip_rc(e != hipSuccess ? e : e2);
}

int dgprf_profile_step(const dgprf_plan_t* plan, const dgprf_chain_t* chain,
                       const dgprf_batch_t* batch, const dgprf_step_t* step, int32_t reps,
                       float* ms_out, void* stream) {
  int rc = check_plan(plan);
  if (!rc) rc = check_chain(chain);
  if (!rc) rc = check_batch(*plan, batch);
  if (!rc) rc = check_step(step);
  if (rc) return rc;
  if (!ms_out || reps < 1) return DGPRF_E_ARG;
  const hipStream_t s = as_stream(stream);
  dgprf_step_t st = *step;
  st.grad_only = 0;
  const UpdateDev ud = make_update_dev(st);
  const int L = plan->n_layers, K = 2 * L + 1;
  // wide first layer (per-layer forward): its A_1 GEMM is timed in a pair of its own, slot K + 1
  const bool ag = plan->a0_off >= 0 && !dgprf_sk::step_fused_fwd(*plan);
  hipEvent_t ev[2 * (2 * DGPRF_MAX_LAYERS + 3)] = {};
  hipError_t e = hipSuccess;
  for (int i = 0; i < 2 * (K + 2) && e == hipSuccess; ++i) e = hipEventCreate(&ev[i]);
  for (int k = 0; k <= K + 1; ++k) ms_out[k] = 0.f;
  // the real step sequence (fwd 0..L-1, bwd L-1..0, update), every kernel between two events
  for (int rep = 0; rep < reps && e == hipSuccess; ++rep) {
    const StepDev sd = make_step_dev(*plan, *chain, *batch, st.step_offset);
    e = dgprf::launch_gather(*plan, sd, s);
    for (int j = 0; j < K && e == hipSuccess; ++j) {
      const int kk = j < L ? j : (j < 2 * L ? L + (2 * L - 1 - j) : 2 * L);
      if (kk == 0 && ag) {
        e = hipEventRecord(ev[2 * (K + 1)], s);
        if (e == hipSuccess) e = dgprf::launch_step_agemm(*plan, sd, s);
        if (e == hipSuccess) e = hipEventRecord(ev[2 * (K + 1) + 1], s);
      }
      if (e == hipSuccess) e = hipEventRecord(ev[2 * kk], s);
      if (e != hipSuccess) break;
      if (kk < L && dgprf_sk::step_fused_fwd(*plan))  // one all-layer forward (timed as layer 0)
        e = kk == 0 ? dgprf::launch_step_fwd_fused(*plan, sd, s) : hipSuccess;
      else if (kk == L - 1 && plan->fold_out)  // folded into the backward: an empty pair
        e = hipSuccess;
      else if (kk < L) e = dgprf::launch_step_fwd(*plan, sd, kk, s, /*with_agemm=*/!ag);
      else if (kk < 2 * L) e = dgprf::launch_step_bwd(*plan, sd, kk - L, s);
      else e = dgprf::launch_step_update(*plan, sd, ud, nullptr, s);
      if (e == hipSuccess) e = hipEventRecord(ev[2 * kk + 1], s);
    }
    if (e == hipSuccess) e = dgprf::launch_advance(chain->step, 1, s);
    if (e == hipSuccess) e = hipEventRecord(ev[2 * K], s);  // empty pair: the pair's own cost
    if (e == hipSuccess) e = hipEventRecord(ev[2 * K + 1], s);
    if (e == hipSuccess) e = hipEventSynchronize(ev[2 * K + 1]);
    for (int kk = 0; kk <= K + (ag ? 1 : 0) && e == hipSuccess; ++kk) {
      float ms = 0.f;
      e = hipEventElapsedTime(&ms, ev[2 * kk], ev[2 * kk + 1]);
      ms_out[kk] += ms / (float)reps;
    }
  }
  for (int i = 0; i < 2 * (K + 2); ++i)
    if (ev[i]) (void)hipEventDestroy(ev[i]);
  return hip_rc(e);
}

int dgprf_forward_scratch(const dgprf_plan_t* plan, int64_t n, int64_t* floats_out) {
  int rc = check_plan(plan);
  if (rc) return rc;
  if (!floats_out || n < 0) return DGPRF_E_ARG;
  *floats_out = dgprf::forward_cfg(*plan, n).scratch_floats;
  return DGPRF_OK;
}

int dgprf_forward(const dgprf_plan_t* plan, const float* theta, const float* omega,
                  const float* der, const float* X, const float* Y, int32_t y_cols, int64_t n,
                  float* const* f_out, float* logp, float* se, float* lse_m, float* lse_s,
                  float* se_sum, float* scratch, int64_t scratch_floats, void* stream) {
  int rc = check_plan(plan);
  if (rc) return rc;
  if (!theta || !omega || !der || n < 0 || (n > 0 && !X)) return DGPRF_E_ARG;
  const bool lik = logp || se || lse_m;
  if (lik && (!Y || y_cols < 1)) return DGPRF_E_ARG;
  if ((lse_m == nullptr) != (lse_s == nullptr)) return DGPRF_E_ARG;
  if (se && plan->likelihood != DGPRF_LIK_GAUSSIAN) return DGPRF_E_ARG;
  if (lik && plan->likelihood == DGPRF_LIK_GAUSSIAN && y_cols < plan->n_gp[plan->n_layers - 1])
    return DGPRF_E_SHAPE;
  if (scratch_floats < 0 || (scratch_floats > 0 && !scratch)) return DGPRF_E_ARG;
  if (scratch_floats < dgprf::forward_cfg(*plan, n).scratch_floats) return DGPRF_E_ARG;
  return hip_rc(dgprf::launch_forward_rows(*plan, theta, omega, der, X, Y, y_cols, n, f_out, logp,
                                           se, lse_m, lse_s, se_sum, scratch, as_stream(stream)));
}

int dgprf_forward_samples(const dgprf_plan_t* plan, const float* thetas, int32_t n_samples,
                          const float* omega, const float* der, const float* X, const float* A1,
                          const float* Y, int32_t y_cols, int64_t n, float* lse_m, float* lse_s,
                          float* se_sum, float* scratch, int64_t scratch_floats, void* stream) {
  int rc = check_plan(plan);
  if (rc) return rc;
  if (!thetas || n_samples < 1 || !omega || !der || n < 0 || (n > 0 && (!X || !Y)) || y_cols < 1 ||
      !lse_m || !lse_s)
    return DGPRF_E_ARG;
  if (se_sum && plan->likelihood != DGPRF_LIK_GAUSSIAN) return DGPRF_E_ARG;
  if (plan->likelihood == DGPRF_LIK_GAUSSIAN && y_cols < plan->n_gp[plan->n_layers - 1])
    return DGPRF_E_SHAPE;
  if (scratch_floats < 0 || (scratch_floats > 0 && !scratch)) return DGPRF_E_ARG;
  // one resident projection serves one Omega_1: not per-chain hyper-parameters over several chains
  if (A1 && plan->hyp_per_chain && plan->n_chains > 1) return DGPRF_E_ARG;
  if (!A1 && scratch_floats < dgprf::forward_cfg(*plan, n).scratch_floats) return DGPRF_E_ARG;
  return hip_rc(dgprf::launch_forward_samples(*plan, thetas, n_samples, omega, der, X, A1, Y, y_cols,
                                              n, lse_m, lse_s, se_sum, scratch, scratch_floats,
                                              as_stream(stream)));
}

int dgprf_forward_samples_scratch(const dgprf_plan_t* plan, int64_t n, int32_t n_samples,
                                  int64_t* floats_out) {
  int rc = check_plan(plan);
  if (rc) return rc;
  if (!floats_out || n < 0 || n_samples < 1) return DGPRF_E_ARG;
  *floats_out = std::max(dgprf::forward_cfg(*plan, n).scratch_floats,
                         dgprf::forward_samples_scratch(*plan, n, n_samples));
  return DGPRF_OK;
}

int dgprf_lse_finalize(const float* lse_m, const float* lse_s, const float* se_sum, int32_t parts,
                       int64_t n, double s_total, float log_y_std, float y_std, float* lse_out,
                       double* out, void* stream) {
  if (!lse_m || !lse_s || !out || parts < 1 || n < 1 || !(s_total > 0.0)) return DGPRF_E_ARG;
  return hip_rc(dgprf::launch_lse_finalize(lse_m, lse_s, se_sum, parts, n, s_total, log_y_std,
                                           y_std, lse_out, out, as_stream(stream)));
}

int dgprf_rf_omega(int32_t kind, int32_t d, int32_t R, const float* z, const float* log_inv_ls,
                   const float* mean, const float* log_amp, float* omega, float* c, void* stream) {
  if ((kind != DGPRF_RBF && kind != DGPRF_ARC) || d < 1 || R < 1) return DGPRF_E_ARG;
  if (!z || !log_inv_ls || !mean || !log_amp || !omega || !c) return DGPRF_E_ARG;
  return hip_rc(dgprf::launch_rf_omega(kind, d, R, z, log_inv_ls, mean, log_amp, omega, c,
                                       as_stream(stream)));
}

int dgprf_rf_features(int32_t kind, const float* X, int64_t n, int32_t d, const float* omega,
                      int32_t R, const float* c, float* phi, void* stream) {
  if ((kind != DGPRF_RBF && kind != DGPRF_ARC) || n < 0 || d < 1 || R < 1) return DGPRF_E_ARG;
  if (!omega || !c || (n > 0 && (!X || !phi))) return DGPRF_E_ARG;
  return hip_rc(dgprf::launch_rf_features(kind, X, n, d, omega, R, c, phi, as_stream(stream)));
}

int dgprf_gp_matmul(const float* phi, int64_t n, int32_t P, const float* W, int32_t g, float* F,
                    void* stream) {
  if (n < 0 || P < 1 || g < 1 || !W || (n > 0 && (!phi || !F))) return DGPRF_E_ARG;
  return hip_rc(dgprf::launch_gp_matmul(phi, n, P, W, g, F, as_stream(stream)));
}

int dgprf_rf_project(const float* X, int64_t n, int32_t ldx, int32_t d, const float* omega,
                     int32_t R, float* A, void* stream) {
  if (n < 0 || d < 1 || R < 1 || ldx < d || !omega || (n > 0 && (!X || !A))) return DGPRF_E_ARG;
  return hip_rc(dgprf::launch_agemm(X, n, ldx, d, omega, R, A, as_stream(stream)));
}

int dgprf_prior_w(const dgprf_plan_t* plan, const float* theta, float* out, void* stream) {
  int rc = check_plan(plan);
  if (rc) return rc;
  if (!theta || !out) return DGPRF_E_ARG;
  return hip_rc(dgprf::launch_prior_w(*plan, theta, out, as_stream(stream)));
}

int dgprf_sghmc_update(const dgprf_plan_t* plan, float* theta, float* mom, const float* grad,
                       const float* mass, const int64_t* step_ctr, uint64_t seed,
                       const dgprf_step_t* step, void* stream) {
  int rc = check_plan(plan);
  if (!rc) rc = check_step(step);
  if (rc) return rc;
  if (!theta || !mom || !grad || !mass || !step_ctr) return DGPRF_E_ARG;
  StepDev sd;
  std::memset(&sd, 0, sizeof(sd));
  sd.theta = theta;
  sd.mom = mom;
  sd.mass = mass;
  sd.step = step_ctr;
  sd.seed = seed;
  sd.step_offset = step->step_offset;
  dgprf_step_t st = *step;
  st.grad_only = 0;
  return hip_rc(dgprf::launch_step_update(*plan, sd, make_update_dev(st), grad, as_stream(stream)));
}

int dgprf_welford_update(const dgprf_plan_t* plan, const float* grad, float* mean, float* m2,
                         int32_t k, int32_t full_bayes, void* stream) {
  int rc = check_plan(plan);
  if (rc) return rc;
  if (!grad || !mean || !m2 || k < 1) return DGPRF_E_ARG;
  return hip_rc(dgprf::launch_welford(*plan, grad, mean, m2, k, full_bayes != 0, as_stream(stream)));
}

int dgprf_mass_estimate(const dgprf_plan_t* plan, const float* mean, const float* m2,
                        int32_t k_batches, int32_t centered, int32_t full_bayes, float* mass_est,
                        float* hmass_est, void* stream) {
  int rc = check_plan(plan);
  if (rc) return rc;
  if (!mean || !m2 || !mass_est || k_batches < 1 || (centered && k_batches < 2)) return DGPRF_E_ARG;
  if (full_bayes && !hmass_est) return DGPRF_E_ARG;
  return hip_rc(dgprf::launch_mass_estimate(*plan, mean, m2, k_batches, centered, full_bayes != 0,
                                            mass_est, hmass_est, as_stream(stream)));
}

}  // extern "C"
