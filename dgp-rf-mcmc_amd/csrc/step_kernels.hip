// step_kernels.hip — the SGHMC/SGLD update, minibatch gather, fresh-z Omega and A_1 GEMM kernels
// of the step, and the host launchers of every step kernel (the forward / backward instances live in
// step_fwd_k*.hip / step_bwd_k*.hip).
//
// Replaces DGP_RF.sgmcmc_update (models/dgp.py:184-216) with full_bayesian=False:
//   forward   per layer l:  Omega_l x -> c*[cos|sin] (RBF) or c*relu (ARC) -> Phi_l W_l
//             (layers/rf_layers.py:29-45,75-91; layers/GP_weight_layers.py:11-15; utils.py:10-44)
//   likelihood + potential U (likelihoods/gaussian.py:18-25, softmax.py:8-15, models/dgp.py:161-182)
//   backward  (analytic form of tape.gradient, models/dgp.py:194-198)
//   update    m <- b m - h N g + sqrt(2(1-b) T M) xi ; theta <- theta + h m / M (models/dgp.py:206-216)
//
// Decomposition (one chain = one blockIdx.z):
//   a workgroup owns a 16-row batch tile x a slice of RF features of one layer; each of its 4 waves
//   owns 16-feature chunks.  Contractions run on v_mfma_f32_16x16x4_f32 (exact fp32):
//     A^T[f][b]  = Omega^T X^T            (K = d_l)
//     F^T[o][b] += W^T Phi^T              (K = features, Phi straight from the A accumulator)
//     gW[f][o]   = Phi^T dF               (K = batch rows; A recomputed in row-major orientation)
//     dPhi[f][b] = W dF^T                 (K = g_l)
//     dX^T[k][b] = Omega dA^T             (K = features)
//   Cross-slice sums of F / dX partials are done by the CONSUMING kernel's prologue: always
//   DGPRF_NS_MAX slices (unused ones are zero) as one unrolled burst of independent loads summed in
//   a fixed order — deterministic, no atomics, one memory round trip.  The gW partials of the row
//   tiles are summed the same way by the update kernel, which also applies the prior term W/N and
//   the SGHMC update with Philox noise.
//
// Latency discipline (this path is latency-bound): every kernel gets a compact
// host-precomputed argument block (one round of independent scalar loads, no plan indexing);
// fragment loads are unconditional with clamped addresses (no exec-masked branches or per-load
// waits) and are issued before the dependent partial sums; minibatch rows of step t+1 are gathered
// by step t's update kernel, so the forward never waits on the step counter or the permutation.
#define DGPRF_STAMPS_TU

#include "step_common.h"

namespace dgprf_sk {
#ifdef DGPRF_STAMPS
unsigned long long* rg_stamp_buffer();
#endif

struct GatherK {
  BatchDev bd;
  const int64_t* step;
  float* xb;  // chain 0 (chain stride ws_cs)
  float* yb;
  float* a0;  // resident A_1 rows (bd.A1): the workspace slab, chain 0
  int64_t ws_cs;
  int32_t B, d_in, yb_cols, step_offset;
  int32_t row_blocks, a1_parts;
};

__global__ void k_gather(const GatherK a) {
  const int chain = blockIdx.y;
  const int64_t t = *a.step + a.step_offset;
  if ((int)blockIdx.x >= a.row_blocks) {  // resident A_1: one wave per (row, part)
    const int w = ((int)blockIdx.x - a.row_blocks) * (int)(blockDim.x >> 6) + (int)(threadIdx.x >> 6);
    const int b = w / a.a1_parts, part = w - b * a.a1_parts;
    if (b < a.B) gather_a1_part(a.bd, a.B, a.a0 + (int64_t)chain * a.ws_cs, chain, t, b, part,
                                threadIdx.x & 63);
    return;
  }
  if (a.d_in > GATHER_WIDE) {  // one wave per row
    const int b = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (b < a.B)
      gather_row_wave(a.bd, a.B, a.d_in, a.yb_cols, a.xb + (int64_t)chain * a.ws_cs,
                      a.yb + (int64_t)chain * a.ws_cs, chain, t, b, threadIdx.x & 63);
    return;
  }
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= a.B) return;
  gather_row(a.bd, a.B, a.d_in, a.yb_cols, a.xb + (int64_t)chain * a.ws_cs,
             a.yb + (int64_t)chain * a.ws_cs, chain, t, b);
}

// Two N(0,1) of counter quad `quad`: words (0,1) (half 0) or (2,3) (half 1) — the same values
// philox_normal4 returns in lanes 2*half, 2*half+1.
__device__ __forceinline__ void philox_normal2(uint64_t seed, uint64_t sub, uint32_t purpose,
                                               uint32_t tag, uint32_t quad, int half, float* z0,
                                               float* z1) {
  u32x4 c;
  c.x = quad;
  c.y = (uint32_t)sub;
  c.z = (uint32_t)(sub >> 32);
  c.w = (purpose << 24) | (tag & 0x00FFFFFFu);
  const u32x4 r = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  box_muller(half ? r.z : r.x, half ? r.w : r.y, z0, z1);
}

typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 ld2(const float* p) { return *reinterpret_cast<const f2*>(p); }
__device__ __forceinline__ void st2(float* p, f2 v) { *reinterpret_cast<f2*>(p) = v; }

// One wave per workgroup, four parameters per lane: the gW partial sums (16 row tiles x 16 bytes
// per lane) are spread over many workgroups instead of concentrated on a few CUs; row tiles
// past n_row_tiles and lanes past w_total lie outside the buffer descriptors (zero, no memory
// traffic), so every load is issued before the first branch.  Specialised on the rarely-used
// paths: GIN (gradient supplied), GONLY (gradient only), XI (injected noise), CYC (cyclical).
constexpr int UPD_THREADS = 64;
__device__ __forceinline__ f2 bload2(rsrc_t r, uint32_t byte_off) {
  return __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(r, byte_off, 0, 0));
}

// One N(0,1) of the hyper-parameter streams (not inlined: the hyper path runs once per step on
// a few CUs, where instruction-cache misses, not arithmetic, set its duration).
__device__ __noinline__ float normal_at(uint64_t seed, uint64_t t, uint32_t purpose, uint32_t chain,
                                        int64_t slot) {
  const f4 z = philox_normal4(seed, t, purpose, chain, (uint32_t)(slot >> 2));
  return z[slot & 3];
}

// Omega elements rebuilt per hyper workgroup (16 per lane)
constexpr int HYP_EPB = UPD_THREADS * 16;

// One hyper workgroup (full_bayesian=True).  The backward left per-workgroup partials
//   [n_rt][NSM][hs]: sum_b X[b][k](dA z^T)[b][k] (k < d), sum_b X[b][k] rowsum(dA)[b], sum dPhi*Phi
// and per row tile the Gaussian lik_log_var term.  Every workgroup of layer l reduces them in the
// same fixed order, forms
//   g_log_amp = sum dPhi*Phi + log_amp/N,   g_lis[k] = exp(lis[k]) sum(...)[k] + lis[k]/N
//   (scalar lis: summed over k),            g_mean[k] = sum_b X[b][k] rowsum(dA)[b] + mean[k]/N
// and applies the SGHMC update of models/dgp.py:206-216 (own momentum, mass and Philox stream) to
// identical new values in LDS; it then rebuilds its HYP_EPB elements of
// Omega_l = exp(lis)[:,None] z_l + mean[:,None] (kernels/RBF.py:43-53, layers/rf_layers.py:34-38).
// The last workgroup of the layer to finish reading the old values (arrival counter, no waiting)
// stores the new hyp / hmom, so no workgroup can read a half-updated set.  Gradient-only mode
// writes dU/d(hyper) into grad_out instead (one workgroup per layer, nothing rebuilt).
template <bool GONLY, bool XI, bool CYC>
__device__ void hyper_block(const UpdK& a, int hb, int chain, float* sm, int sb) {
  const HypK& k = a.hk;
  const int tid = threadIdx.x, L = a.n_layers;
  constexpr int NT = UPD_THREADS;
  float* hyp = k.hyp + (int64_t)chain * k.hyp_cs;
  float* hm = k.hmom + (int64_t)chain * k.hyp_total;
  const float* hmass = k.hmass + chain * DGPRF_HMASS;
  float* gout = a.grad_out + (int64_t)chain * a.grad_cs + a.w_total;
  const UpdateDev& ud = a.ud;
  const float N = ud.data_size;
  const int64_t t = *a.step + (int64_t)a.step_offset;
  float lr, T;
  int resample;
  step_schedule<CYC>(ud, t, &lr, &T, &resample);
  const float h = sqrtf(lr / N), beta = ud.beta;
  // SGHMC update of hyper slot `slot` (value v, momentum m, mass slot midx); returns the new value
  auto upd = [&](int64_t slot, float g, float v, float m, int midx, float* m_out) -> float {
    if (GONLY) {
      gout[slot] = g;
      return v;
    }
    const float M = hmass[midx];
    if (resample)
      m = (XI && ud.xi_hyp_resample)
              ? ud.xi_hyp_resample[(int64_t)chain * k.hyp_total + slot]
              : normal_at(a.seed, (uint64_t)t, DGPRF_RNG_HYPER_RESAMPLE, chain, slot);
    const float eps = (XI && ud.xi_hyp) ? ud.xi_hyp[(int64_t)chain * k.hyp_total + slot]
                                        : normal_at(a.seed, (uint64_t)t, DGPRF_RNG_HYPER, chain, slot);
    const float mn = beta * m - (h * N) * g + sqrtf(2.0f * (1.0f - beta) * T * M) * eps;
    *m_out = mn;
    return v + (h * (1.0f / M)) * mn;
  };
  if (hb == k.n_blocks - 1) {  // Gaussian lik_log_var (likelihoods/gaussian.py:12)
    const bool lik_tr = (k.flags & DGPRF_HYP_LIK) && k.likelihood == DGPRF_LIK_GAUSSIAN;
    if (GONLY) {  // slots no workgroup owns (padding, groups that do not train) read as 0
      for (int64_t s = tid; s < k.hyp_total; s += NT) {
        bool owned = s < L ? (k.flags & DGPRF_HYP_KERNEL) != 0 : (s == L && lik_tr);
        for (int q = 0; q < L; ++q) {
          owned |= (k.flags & DGPRF_HYP_KERNEL) && s >= k.lis_off[q] && s < k.lis_off[q] + k.d[q];
          owned |= (k.flags & DGPRF_HYP_MEAN) && s >= k.mean_off[q] && s < k.mean_off[q] + k.d[q];
        }
        if (!owned) gout[s] = 0.f;
      }
    }
    if (lik_tr && tid == 0) {
      const float* hpl = k.ws + (int64_t)chain * a.ws_cs + k.hpl_off;
      float s = 0.f;
      for (int rt = 0; rt < a.n_rt; ++rt) s += hpl[rt];
      const float v0 = hyp[L];
      float mn = 0.f;
      const float v = upd(L, s + v0 / N, v0, GONLY ? 0.f : hm[L], 24, &mn);
      if (!GONLY) {
        hm[L] = mn;
        hyp[L] = v;
        k.der[(int64_t)chain * k.der_cs + DGPRF_MAX_LAYERS] = expf(v);
      }
    }
    return;
  }
  int l = 0;
  for (int q = 1; q < L; ++q)
    if (hb >= k.b0[q]) l = q;
  // uniform by construction; through readfirstlane so the partial-row descriptor below is built in
  // SGPRs (otherwise each of its loads is a waterfall loop)
  l = __builtin_amdgcn_readfirstlane(l);
  const int j = hb - k.b0[l], d = k.d[l], R = k.R[l], nv = 2 * d + 1, hs = (nv + 3) & ~3;
  const int Q = hs >> 2, ns = k.ns[l], P = a.n_rt * ns, RG = Q >= NT ? 1 : NT / Q;
  const bool kern = (k.flags & DGPRF_HYP_KERNEL) != 0, mean = (k.flags & DGPRF_HYP_MEAN) != 0;
  const int64_t lis = k.lis_off[l], mo = k.mean_off[l];
  // LDS: totals | old values | old momenta | new values | exp(new lis) | row-group partials | tree
  float* tot = sm;
  float* ov = tot + hs;   // [0] log_amp, [1+k] log_inv_ls, [1+d+k] mean
  float* om = ov + hs;
  float* nvv = om + hs;
  float* els = nvv + hs;  // exp(new lis)[d]
  float* part = els + hs;                       // [RG][hs]
  float* red = part + (4 * NT > hs ? 4 * NT : hs);  // [NT] tree, [NT] last-arrival flag
  auto slot_of = [&](int e) -> int64_t { return e == 0 ? (int64_t)l : (e <= d ? lis + e - 1 : mo + e - 1 - d); };
  // (0) z of this workgroup's Omega slice and the old values / momenta first: independent loads
  float* omg = k.omega + (int64_t)chain * k.om_cs + k.om_off[l];
  const int64_t n_el = (int64_t)d * R, base = (int64_t)j * HYP_EPB;
  f4 zv[4];
  if (!GONLY) {
    const rsrc_t rz = make_rsrc_u(k.z + k.om_off[l], (int)n_el);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t i = base + 4 * (tid + NT * u);
      zv[u] = bload4(rz, i < n_el ? (uint32_t)(i * 4) : DGPRF_OOB);
    }
  }
  for (int e = tid; e < 1 + 2 * d; e += NT) {
    const int64_t s = slot_of(e);
    ov[e] = hyp[s];
    om[e] = GONLY ? 0.f : hm[s];
  }
  __syncthreads();  // every old value of this workgroup has been read
  DGPRF_STAMP(sb, 1);
  // arrival on the layer's counter (its return overlaps the partial loads below)
  unsigned* cnt = reinterpret_cast<unsigned*>(const_cast<float*>(k.ws) + (int64_t)chain * a.ws_cs +
                                              k.cnt_off) + l;
  unsigned arrived = 0u;
  if (!GONLY && k.nb[l] > 1 && tid == 0) arrived = atomicAdd(cnt, 1u);
  // (1) partial row sums: up to HYP_U loads per lane in flight, summed in row order
  // rows p = rt * ns + sl of a row group advance by RG: (rt, sl) tracked without divisions
  constexpr int HYP_U = 8;
  const float* hp = k.ws + (int64_t)chain * a.ws_cs + k.hpp_off[l];
  const rsrc_t rh = make_rsrc_u(hp, a.n_rt * NSM * hs);
  const int st_rt = RG / ns, st_sl = RG - st_rt * ns;
  for (int i = tid; i < RG * Q; i += NT) {
    const int q = i % Q, rg = i / Q;
    int rt = rg / ns, sl = rg - rt * ns;
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int p0 = rg; p0 < P; p0 += HYP_U * RG) {
      f4 v[HYP_U];
#pragma unroll
      for (int u = 0; u < HYP_U; ++u) {
        v[u] = bload4(rh, rt < a.n_rt ? (uint32_t)(((rt * NSM + sl) * hs + 4 * q) * 4) : DGPRF_OOB);
        rt += st_rt;
        sl += st_sl;
        if (sl >= ns) {
          sl -= ns;
          ++rt;
        }
      }
#pragma unroll
      for (int u = 0; u < HYP_U; ++u) acc += v[u];
    }
    *reinterpret_cast<f4*>(part + rg * hs + 4 * q) = acc;
  }
  DGPRF_STAMP(sb, 2);
  __syncthreads();
  for (int e = tid; e < nv; e += NT) {
    float s = 0.f;
    for (int rg = 0; rg < RG; ++rg) s += part[rg * hs + e];
    tot[e] = s;
  }
  __syncthreads();
  DGPRF_STAMP(sb, 3);
  // (2) new values: one update site for every slot (scalar lis: one slot, broadcast after)
  const bool scalar_lis = kern && !k.ard[l];
  float gsc = 0.f;
  if (scalar_lis) {  // one length scale: its gradient sums over the d dims (fixed-order tree)
    float sp = 0.f;
    for (int kk = tid; kk < d; kk += NT) sp += expf(ov[1 + kk]) * tot[kk];
    red[tid] = sp;
    __syncthreads();
    for (int w = NT / 2; w > 0; w >>= 1) {
      if (tid < w) red[tid] += red[tid + w];
      __syncthreads();
    }
    gsc = red[0];
  }
  for (int e = tid; e < 1 + 2 * d; e += NT) {
    float v = ov[e], mn = om[e];
    bool tr;
    float g;
    int midx;
    int64_t slot;
    if (e == 0) {
      tr = kern;
      g = tot[2 * d];
      midx = l;
      slot = l;
    } else if (e <= d) {
      tr = kern && (!scalar_lis || e == 1);
      g = scalar_lis ? gsc : expf(ov[e]) * tot[e - 1];
      midx = 8 + l;
      slot = lis + e - 1;
    } else {
      tr = mean;
      g = tot[e - 1];
      midx = 16 + l;
      slot = mo + e - 1 - d;
    }
    if (tr) v = upd(slot, g + ov[e] / N, ov[e], om[e], midx, &mn);
    nvv[e] = v;
    om[e] = mn;
  }
  if (scalar_lis) {
    __syncthreads();
    for (int kk = 1 + tid; kk < d; kk += NT) {
      nvv[1 + kk] = nvv[1];
      om[1 + kk] = om[1];
      if (GONLY) gout[lis + kk] = gsc + ov[1] / N;
    }
  }
  if (GONLY) return;
  __syncthreads();
  DGPRF_STAMP(sb, 4);
  for (int kk = tid; kk < d; kk += NT) els[kk] = expf(nvv[1 + kk]);
  // (3) the last workgroup of the layer to arrive stores the new hyp / hmom
  bool last = k.nb[l] == 1;
  if (!last) {
    if (tid == 0) {
      const bool lst = arrived == (unsigned)k.nb[l] - 1u;
      if (lst) *cnt = 0u;
      red[NT] = lst ? 1.f : 0.f;
    }
    __syncthreads();
    last = red[NT] != 0.f;
  } else {
    __syncthreads();
  }
  if (last) {
    for (int e = tid; e < 1 + 2 * d; e += NT) {
      const bool tr = e == 0 ? kern : (e <= d ? kern : mean);
      if (!tr) continue;
      const int64_t s = slot_of(e);
      hyp[s] = nvv[e];
      hm[s] = om[e];
    }
  }
  DGPRF_STAMP(sb, 5);
  // (4) this workgroup's slice of Omega_l and c_l (layers/rf_layers.py:44,90)
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int64_t i = base + 4 * (tid + NT * u);
    if (i >= n_el) continue;
    f4 o;
    int kk = (int)((uint32_t)i / (uint32_t)R), rc = (int)i - kk * R;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int kc = kk < d ? kk : d - 1;
      o[c] = els[kc] * zv[u][c] + nvv[1 + d + kc];
      for (++rc; rc >= R; rc -= R) ++kk;
    }
    if (i + 3 < n_el) {
      *reinterpret_cast<f4*>(omg + i) = o;
    } else {
      for (int c = 0; c < 4 && i + c < n_el; ++c) omg[i + c] = o[c];
    }
  }
  if (j == 0 && tid == 0) {
    const float amp = expf(nvv[0]), sq = sqrtf((float)R);
    k.der[(int64_t)chain * k.der_cs + l] = k.kind[l] == DGPRF_RBF ? amp / sq : (sqrtf(2.f) * amp) / sq;
  }
#ifdef DGPRF_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  DGPRF_STAMP(sb, 14);
}

template <bool GIN, bool GONLY, bool XI, bool CYC>
__device__ __forceinline__ void update_block(const UpdK& a, float* usm) {
  const int chain = blockIdx.y;
  const int stamp_base = 16 * 4096 + blockIdx.y * gridDim.x + blockIdx.x;
  DGPRF_STAMP(stamp_base, 0);
  if (!GIN && (int)blockIdx.x < a.hyp_blocks) {  // full_bayesian=True hyper-parameters
    hyper_block<GONLY, XI, CYC>(a, (int)blockIdx.x, chain, usm, stamp_base);
    return;
  }
  const int bx = (int)blockIdx.x - a.hyp_blocks;
  if (bx >= a.upd_blocks + a.gather_blocks) {  // resident A_1 rows of step t+1: (row, part) each
    const int64_t t = *a.step + (int64_t)a.step_offset;
    const int w = bx - a.upd_blocks - a.gather_blocks;
    const int b = w / a.a1_parts, part = w - b * a.a1_parts;
    if (b < a.B) gather_a1_part(a.bd, a.B, a.a0 + (int64_t)chain * a.ws_cs, chain, t + 1, b, part,
                                threadIdx.x);
    return;
  }
  if (bx >= a.upd_blocks) {  // dedicated blocks: rows of step t+1 (off the path)
    const int64_t t = *a.step + (int64_t)a.step_offset;
    if (a.d_in > GATHER_WIDE) {  // one-wave blocks: one row each
      const int b = bx - a.upd_blocks;
      if (a.gather_next && b < a.B)
        gather_row_wave(a.bd, a.B, a.d_in, a.yb_cols, a.xb + (int64_t)chain * a.ws_cs,
                        a.yb + (int64_t)chain * a.ws_cs, chain, t + 1, b, threadIdx.x);
      return;
    }
    const int b = (bx - a.upd_blocks) * UPD_THREADS + threadIdx.x;
    if (a.gather_next && b < a.B)
      gather_row(a.bd, a.B, a.d_in, a.yb_cols, a.xb + (int64_t)chain * a.ws_cs,
                 a.yb + (int64_t)chain * a.ws_cs, chain, t + 1, b);
    return;
  }
  // four packed parameters per lane
  w_update_quad<GIN, GONLY, XI, CYC>(a, 4 * (bx * UPD_THREADS + (int)threadIdx.x), chain);
#ifdef DGPRF_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  DGPRF_STAMP(stamp_base, 14);
}

template <bool GIN, bool GONLY, bool XI, bool CYC>
__global__ __launch_bounds__(UPD_THREADS) void k_step_update(const UpdK a) {
  extern __shared__ __attribute__((aligned(16))) float usm[];
  update_block<GIN, GONLY, XI, CYC>(a, usm);
  // eager steps (adv_cnt set): the last workgroup to finish advances the step counter — the
  // launch of k_advance a graph makes once per replay.  Every workgroup has consumed its read of
  // the counter before it arrives, so none of them sees the new value.
  if (a.adv_cnt) {
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned total = gridDim.x * gridDim.y;
      if (atomicAdd(a.adv_cnt, 1u) == total - 1u) {
        atomicExch(a.adv_cnt, 0u);
        atomicAdd(reinterpret_cast<unsigned long long*>(a.step_adv), 1ull);
      }
    }
  }
}


// random_fixed=False (layers/rf_layers.py:39-41): Omega_l = exp(lis_l)[:,None] z + mean_l[:,None]
// with z ~ N(0,1) drawn for this step — Philox (seed, sub = step, DGPRF_RNG_Z, tag = 1 + l + 16
// chain), element i of the layer at counter quad i / 4 — for the fresh layers.  One thread per
// 4 elements; chain blockIdx.y writes its own workspace copy.  copy_fixed (the all-layer fused
// forward reads every layer from this copy): the other layers' Omega is copied in from the
// chain's Omega (chain stride om_cs), so the copy is the whole step's Omega.
__global__ void k_fresh_omega(const dgprf_plan_t pl, const float* __restrict__ hyp, float* ws,
                              const int64_t* step, uint64_t seed, int32_t step_offset,
                              const float* __restrict__ omega, int64_t om_cs, int32_t copy_fixed) {
  const int chain = blockIdx.y;
  const int64_t i0 = 4 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  if (i0 >= pl.omega_total) return;
  int layer = 0;
  for (int l = 1; l < pl.n_layers; ++l)
    if (i0 >= pl.omega_off[l]) layer = l;
  float* om = ws + (int64_t)chain * pl.ws_chain + pl.omf_off;
  const int64_t n_l = (int64_t)pl.d[layer] * pl.n_rf[layer];
  const int64_t j0 = i0 - pl.omega_off[layer];  // omega_off is a multiple of 4
  if (!((pl.fresh_z >> layer) & 1)) {
    if (copy_fixed) {
      const float* src = omega + (int64_t)chain * om_cs;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (j0 + c < n_l) om[i0 + c] = src[i0 + c];
    }
    return;
  }
  const float* h = hyp + (pl.hyp_per_chain ? (int64_t)chain * pl.hyp_total : 0);
  const int64_t t = *step + step_offset;
  const f4 z = philox_normal4(seed, (uint64_t)t, DGPRF_RNG_Z, 1u + layer + 16u * chain,
                              (uint32_t)(j0 >> 2));
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int64_t j = j0 + c;
    if (j < n_l) {
      const int k = (int)(j / pl.n_rf[layer]);
      om[pl.omega_off[layer] + j] = expf(h[pl.lis_off[layer] + k]) * z[c] + h[pl.mean_off[layer] + k];
    }
  }
}

__global__ void k_advance(int64_t* step, int64_t by) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *step += by;
}

// ------------------------------------------------------------------------- wide first layer
// A_1 = X Omega_1 for a first layer with d > 32 (BASELINE config 4: d = 784, R = 4096), written
// to the workspace for the layer-0 forward and backward, which would otherwise each run a d-long
// dependent k-step loop per 16-feature chunk.  One workgroup = 32 rows x 64 features; its 4 waves
// own 16 x 32 sub-tiles (2 accumulators); K runs in LDS-staged blocks of 32 (X block [32][33],
// Omega block [32][68]), the next block's loads in flight while the current one computes.  Rows
// >= B and k >= d are staged as zeros.
struct AgemmK {
  const float* xrows;  // [B][d_in] of chain 0 (stride xrow_cs)
  const float* om;     // Omega_1 [d][R] of chain 0 (stride om_cs)
  float* aout;         // [align32(B)][R] of chain 0 (stride ws_cs)
  int64_t xrow_cs, om_cs, ws_cs;
  int32_t B, d, R, d_in;
  int32_t n_out, pad;  // rows of aout written (>= B; rows >= B are zeros)
};
constexpr int AG_KB = 32, AG_XST = 33, AG_OST = 68;

__global__ __launch_bounds__(256) void k_step_agemm(const AgemmK a) {
  __shared__ float xsm[2][32 * AG_XST];
  __shared__ __attribute__((aligned(16))) float osm[2][AG_KB * AG_OST];
  const int chain = blockIdx.z;
  const int rb = blockIdx.y * 32, fb = blockIdx.x * 64;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 15, lq = lane >> 4;
  const int wr = wave >> 1, wc = wave & 1;
  const float* X = a.xrows + (int64_t)chain * a.xrow_cs;
  const float* om = a.om + (int64_t)chain * a.om_cs;
  const int d = a.d, R = a.R;
  // staging assignment: X block: 4 scalars per thread (row tid >> 3, k (tid & 7) * 4 + q);
  // Omega block: 2 float4 per thread (k = e >> 4, features 4 (e & 15))
  const int xr = tid >> 3, xk = (tid & 7) * 4;
  const rsrc_t rx = make_rsrc(X, (int64_t)a.B * a.d_in);
  const rsrc_t ro = make_rsrc(om, (int64_t)d * R);
  float xv[4];
  f4 ov[2];
  auto load = [&](int kb) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = rb + xr, k = kb + xk + q;
      xv[q] = bload1(rx, row < a.B && k < d ? (uint32_t)(((int64_t)row * a.d_in + k) * 4) : DGPRF_OOB);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int e = tid + 256 * j, k = kb + (e >> 4), f = fb + 4 * (e & 15);
      ov[j] = bload4(ro, k < d && f < R ? (uint32_t)(((int64_t)k * R + f) * 4) : DGPRF_OOB);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 4; ++q) xsm[buf][xr * AG_XST + xk + q] = xv[q];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int e = tid + 256 * j;
      *reinterpret_cast<f4*>(&osm[buf][(e >> 4) * AG_OST + 4 * (e & 15)]) = ov[j];
    }
  };
  f4 acc0 = f4zero(), acc1 = f4zero();
  const int nkb = (d + AG_KB - 1) / AG_KB;
  load(0);
  store(0);
  __syncthreads();
  for (int kb = 0; kb < nkb; ++kb) {
    const int buf = kb & 1;
    if (kb + 1 < nkb) load((kb + 1) * AG_KB);
    const float* xb = &xsm[buf][(wr * 16 + lr) * AG_XST + lq];
    const float* ob = &osm[buf][lq * AG_OST + wc * 32 + lr];
#pragma unroll
    for (int ks = 0; ks < AG_KB / 4; ++ks) {
      const float xa = xb[4 * ks];
      acc0 = mfma16(xa, ob[4 * ks * AG_OST], acc0);
      acc1 = mfma16(xa, ob[4 * ks * AG_OST + 16], acc1);
    }
    if (kb + 1 < nkb) store(buf ^ 1);
    __syncthreads();
  }
  // acc[r] = A[row wr*16 + 4lq + r][feature wc*32 + n*16 + lr]
  float* out = a.aout + (int64_t)chain * a.ws_cs;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t row = rb + wr * 16 + 4 * lq + r;
    const int f = fb + wc * 32 + lr;
    if (row >= a.n_out) continue;
    if (f < R) out[row * R + f] = acc0[r];
    if (f + 16 < R) out[row * R + f + 16] = acc1[r];
  }
}

void k_step_fwd_launch(int d, int g, bool rbf, int nw, dim3 grid, size_t lds, hipStream_t s,
                       const LayerK& a) {
  if (d <= 4) k_step_fwd_launch2<1>(g, rbf, nw, grid, lds, s, a);
  else if (d <= 8) k_step_fwd_launch2<2>(g, rbf, nw, grid, lds, s, a);
  else if (d <= 16) k_step_fwd_launch2<4>(g, rbf, nw, grid, lds, s, a);
  else if (d <= 32) k_step_fwd_launch2<8>(g, rbf, nw, grid, lds, s, a);
  else k_step_fwd_launch2<0>(g, rbf, nw, grid, lds, s, a);
}

void k_step_bwd_launch(int d, int g, bool rbf, bool fb, bool w8, dim3 grid, size_t lds,
                       hipStream_t s, const LayerK& a) {
  if (d <= 4) k_step_bwd_launch2<1>(g, rbf, fb, w8, grid, lds, s, a);
  else if (d <= 8) k_step_bwd_launch2<2>(g, rbf, fb, w8, grid, lds, s, a);
  else if (d <= 16) k_step_bwd_launch2<4>(g, rbf, fb, w8, grid, lds, s, a);
  else if (d <= 32) k_step_bwd_launch2<8>(g, rbf, fb, w8, grid, lds, s, a);
  else k_step_bwd_launch2<0>(g, rbf, fb, w8, grid, lds, s, a);
}

}  // namespace dgprf_sk

using namespace dgprf_sk;

#ifdef DGPRF_STAMPS
// row-group backward stamps: a buffer of their own (17 x 4096 bases x 16 slots)
static unsigned long long* g_rg_stamps = nullptr;
unsigned long long* dgprf_sk::rg_stamp_buffer() {
  if (!g_rg_stamps && hipMalloc(&g_rg_stamps, (size_t)17 * 4096 * 16 * 8) == hipSuccess)
    (void)hipMemset(g_rg_stamps, 0, (size_t)17 * 4096 * 16 * 8);
  return g_rg_stamps;
}
extern "C" int dgprf_debug_read_rg_stamps(unsigned long long* host, long long n) {
  return g_rg_stamps && hipMemcpy(host, g_rg_stamps, (size_t)n * 8, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -3;
}
__device__ unsigned long long g_dgprf_stamps[17 * 4096 * DGPRF_STAMP_SLOTS];
extern "C" int dgprf_debug_read_stamps(unsigned long long* host, long long n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_dgprf_stamps), (size_t)n * 8, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : -3;
}
extern "C" int dgprf_debug_clear_stamps(void) {
  static unsigned long long zeros[17 * 4096 * DGPRF_STAMP_SLOTS];
  if (g_rg_stamps) (void)hipMemset(g_rg_stamps, 0, (size_t)17 * 4096 * 16 * 8);
  return hipMemcpyToSymbol(HIP_SYMBOL(g_dgprf_stamps), zeros, sizeof(zeros), 0,
                           hipMemcpyHostToDevice) == hipSuccess ? 0 : -3;
}
#endif

namespace dgprf {

// A_1 = X Omega_1 of the step's gathered rows into the workspace (plan.a0_off).
hipError_t launch_step_agemm(const dgprf_plan_t& pl, const StepDev& sd, hipStream_t s) {
  int lds_floats = 0;
  const LayerK a = make_layer_k(pl, sd, 0, lds_floats);
  if (!a.a0) return hipSuccess;
  hipError_t err = hipSuccess;
  const int64_t rows = (pl.batch + 31) / 32 * 32;  // the [align32(B)][R] buffer, zero-padded
  // the hand-written MFMA GEMM (agemm.hip); k_step_agemm for shapes outside it
  if (own_agemm(a.xrows, pl.batch, rows, pl.d_in, pl.d[0], a.om, pl.n_rf[0], sd.ws + pl.a0_off,
                pl.n_chains, a.xrow_cs, a.om_cs, pl.ws_chain, a.a0_sl ? 2 : 1, a.a0_sl, s, &err))
    return err;
  AgemmK g;
  g.xrows = a.xrows;
  g.om = a.om;
  g.aout = sd.ws + pl.a0_off;
  g.xrow_cs = a.xrow_cs;
  g.om_cs = a.om_cs;
  g.ws_cs = pl.ws_chain;
  g.B = pl.batch;
  g.d = pl.d[0];
  g.R = pl.n_rf[0];
  g.d_in = pl.d_in;
  g.n_out = (int32_t)rows;
  g.pad = 0;
  dim3 ggrid((unsigned)((g.R + 63) / 64), (unsigned)((g.B + 31) / 32), pl.n_chains);
  hipLaunchKernelGGL(k_step_agemm, ggrid, dim3(256), 0, s, g);
  return hipGetLastError();
}

hipError_t launch_step_fwd(const dgprf_plan_t& pl, const StepDev& sd, int layer, hipStream_t s,
                           bool with_agemm) {
  // 8 waves per workgroup when every wave still gets >= 2 chunks (config 3, cpw = 2: one chunk
  // per wave measured slower, 37.6 vs 35.9 us/step)
  const bool w8 = pl.cpw[layer] >= 4 && pl.cpw[layer] % 2 == 0;
  // 16 waves (four per SIMD) when every wave still gets >= 2 chunks (config 5, cpw = 8:
  // 104.4 -> 102.4 us/step; with one chunk per wave, config 4, no gain)
  const int nwf = (w8 && pl.cpw[layer] % 8 == 0) ? 16 : (w8 ? 8 : 4);
  int lds_floats = 0;
  LayerK a = make_layer_k(pl, sd, layer, lds_floats, false, nwf);
#ifdef DGPRF_STAMPS
  a.stamps = rg_stamp_buffer();
#endif
  // wide first layer: A_1 = X Omega_1 first — unless the rows were gathered from the dataset's
  // resident projection (sd.bd.A1)
  if (a.a0 && with_agemm && !sd.bd.A1) {
    const hipError_t e = launch_step_agemm(pl, sd, s);
    if (e != hipSuccess) return e;
  }
  dim3 grid(a.main_blocks, 1, pl.n_chains);
  k_step_fwd_launch(pl.d[layer], pl.n_gp[layer], pl.kind[layer] == DGPRF_RBF, nwf, grid,
                    (size_t)lds_floats * sizeof(float), s, a);
  return hipGetLastError();
}

hipError_t launch_step_fwd_fused(const dgprf_plan_t& pl, const StepDev& sd, hipStream_t s) {
  if (!step_fused_fwd(pl)) return hipErrorInvalidValue;
  float* f_out[DGPRF_MAX_LAYERS];
  for (int l = 0; l < DGPRF_MAX_LAYERS; ++l) f_out[l] = l < pl.n_layers ? sd.ws + pl.fp_off[l] : nullptr;
  const bool direct = sd.bd.mode == DGPRF_BATCH_DIRECT;
  const float* X = direct ? sd.bd.X : sd.ws + pl.xb_off;
  // random_fixed=False layers: this step's Omega is the workspace copy (k_fresh_omega)
  const float* om = pl.fresh_z && pl.omf_off >= 0 ? sd.ws + pl.omf_off : sd.omega;
  return launch_forward_rows(pl, sd.theta, om, sd.der, X, nullptr, 0, pl.batch, f_out, nullptr,
                             nullptr, nullptr, nullptr, nullptr, nullptr, s);
}

hipError_t launch_step_bwd(const dgprf_plan_t& pl, const StepDev& sd, int layer, hipStream_t s) {
  RwCfg w;
  if (pl.rt_per_group > 1 && pl.ws_chain >= (int64_t)1 << 29)
    return hipErrorInvalidValue;  // 32-bit buffer offsets of the row-group / row-wave kernels
  if (pl.rt_per_group > 1 && rw_config(pl, layer, sd.full_bayes != 0, w)) {
    // row-wave backward (narrow slices after the fused forward): no barrier in the row-tile loop
    int lds_floats = 0;
    LayerK a = make_layer_k(pl, sd, layer, lds_floats, /*bwd=*/true, 4);
    set_block_map(a, pl.n_gw_rows, pl.n_chains);
    a.rt_per_rg = pl.rt_per_group;
    a.cmp = 1;
    a.rw_one = a.last;
    a.wsa_off = w.wsa;
    a.osa_off = w.osa;
    a.osa_st = w.ost;
    a.aux_off = w.wave0;    // wave-private X / dF / Y tiles at aux_off + wave * red_off
    a.red_off = w.wstride;
    a.auxst = w.dst;  // zero-padded wave tiles (rw_config)
    a.xst = w.xst;
    a.rw_orows = w.orows;
    a.hred_off = w.hred;
    a.gred_off = w.gred;
    a.dsrc_off = a.last ? (int)pl.fp_off[layer] : (layer + 1 < pl.n_layers ? (int)pl.dxp_off[layer + 1] : 0);
#ifdef DGPRF_STAMPS
    a.stamps = rg_stamp_buffer();
#endif
    dim3 grid(a.main_blocks, 1, pl.n_chains);
    const int d = pl.d[layer], g = pl.n_gp[layer];
    const bool rbf = pl.kind[layer] == DGPRF_RBF, fb = sd.full_bayes != 0;
    const size_t lds = (size_t)w.total * sizeof(float);
    if (d <= 4) k_step_bwd_rw_launch2<1>(g, rbf, fb, layer > 0, w.nch, w.nwv, grid, lds, s, a);
    else if (d <= 8) k_step_bwd_rw_launch2<2>(g, rbf, fb, layer > 0, w.nch, w.nwv, grid, lds, s, a);
    else if (d <= 16) k_step_bwd_rw_launch2<4>(g, rbf, fb, layer > 0, w.nch, w.nwv, grid, lds, s, a);
    else k_step_bwd_rw_launch2<8>(g, rbf, fb, layer > 0, w.nch, w.nwv, grid, lds, s, a);
    return hipGetLastError();
  }
  if (pl.rt_per_group > 1) {  // row-group backward: at most 16 gW partial rows whatever B
    RgCfg c;
    if (!rg_config(pl, layer, sd.full_bayes != 0, c)) return hipErrorInvalidValue;
    int lds_floats = 0;
    LayerK a = make_layer_k(pl, sd, layer, lds_floats, /*bwd=*/true, 4);
    set_block_map(a, pl.n_gw_rows, pl.n_chains);
    a.rt_per_rg = pl.rt_per_group;
    a.ncw = c.ncw;
    a.nrw = c.nrw;
    a.rg_nit = c.nit;
    a.rg_fast = c.fast;
    a.aux_off = c.aux;
    a.red_off = c.red;
    a.wsa_off = c.wsa;
    a.osa_off = c.osa;
    a.osa_st = c.ost;
    a.hred_off = c.hred;
    a.gred_off = c.gred;
    a.cmp = step_fused_fwd(pl) ? 1 : 0;
#ifdef DGPRF_STAMPS
    a.stamps = rg_stamp_buffer();
#endif
    dim3 grid(a.main_blocks, 1, pl.n_chains);
    const int d = pl.d[layer], g = pl.n_gp[layer];
    const bool rbf = pl.kind[layer] == DGPRF_RBF, fb = sd.full_bayes != 0;
    const size_t lds = (size_t)c.total * sizeof(float);
    if (d <= 4) k_step_bwd_rg_launch2<1>(g, rbf, fb, c.nit, grid, lds, s, a);
    else if (d <= 8) k_step_bwd_rg_launch2<2>(g, rbf, fb, c.nit, grid, lds, s, a);
    else if (d <= 16) k_step_bwd_rg_launch2<4>(g, rbf, fb, c.nit, grid, lds, s, a);
    else if (d <= 32) k_step_bwd_rg_launch2<8>(g, rbf, fb, c.nit, grid, lds, s, a);
    else k_step_bwd_rg_launch2<0>(g, rbf, fb, c.nit, grid, lds, s, a);
    return hipGetLastError();
  }
  // 8 waves per workgroup for W-only steps whose slices are staged whole (a.wstage); a folded
  // output layer runs the 4-wave instance that recomputes F_L
  const bool fold = pl.fold_out && !sd.full_bayes && layer == pl.n_layers - 1;
  bool w8 = !sd.full_bayes && pl.cpw[layer] % 4 == 0 && !fold;
  int lds_floats = 0;
  LayerK a = make_layer_k(pl, sd, layer, lds_floats, /*bwd=*/true, w8 ? 8 : 4);
  if (w8 && !a.wstage) {  // the slice image does not fit next to 8 waves' rows: 4 waves
    w8 = false;
    lds_floats = 0;
    a = make_layer_k(pl, sd, layer, lds_floats, /*bwd=*/true, 4);
  }
  // the step launched no forward for a folded output layer: its backward must recompute F_L
  if (fold && !(a.rcf && a.fast)) return hipErrorInvalidValue;
#ifdef DGPRF_STAMPS
  a.stamps = rg_stamp_buffer();
#endif
  dim3 grid(a.main_blocks, 1, pl.n_chains);
  k_step_bwd_launch(pl.d[layer], pl.n_gp[layer], pl.kind[layer] == DGPRF_RBF, sd.full_bayes != 0,
                    w8, grid, (size_t)lds_floats * sizeof(float), s, a);
  return hipGetLastError();
}

hipError_t launch_step_update(const dgprf_plan_t& pl, const StepDev& sd, const UpdateDev& ud,
                              const float* grad_in, hipStream_t s, bool gather_next,
                              bool advance) {
  if (pl.w_total >= (int64_t)1 << 30 ||
      (int64_t)pl.n_rt_pad * gw_row_stride(pl.w_total) >= (int64_t)1 << 29)
    return hipErrorInvalidValue;  // 32-bit buffer offsets
  UpdK a;
  a.theta = sd.theta;
  a.mom = sd.mom;
  a.gwp = sd.ws ? sd.ws + pl.gwp_off : nullptr;
  a.mass = sd.mass;
  a.step = sd.step;
  a.w_total = (int32_t)pl.w_total;
  a.gw_ld = (int32_t)gw_row_stride(pl.w_total);
  a.pad_g = 0;
  a.n_rt = pl.n_gw_rows;  // gW partial rows (one per row tile, or per row group)
  a.n_rt_pad = pl.n_rt_pad;
  a.n_layers = pl.n_layers;
  for (int l = 0; l < DGPRF_MAX_LAYERS; ++l) {
    a.lo[l] = l < pl.n_layers ? (int32_t)pl.w_off[l] : INT32_MAX;
    a.hi[l] = l < pl.n_layers ? (int32_t)(pl.w_off[l] + (int64_t)pl.P[l] * pl.n_gp[l]) : 0;
  }
  a.seed = sd.seed;
  a.ws_cs = pl.ws_chain;
  a.step_offset = sd.step_offset;
  a.ud = ud;
  a.grad_in = grad_in;
  a.grad_out = sd.grad_out;
  a.grad_cs = pl.w_total + (sd.full_bayes ? pl.hyp_total : 0);
  a.e_end = a.hi[pl.n_layers - 1];
  a.pad_e = 0;
  a.gather_next = gather_next && sd.bd.mode == DGPRF_BATCH_EPOCH ? 1 : 0;
  // the step-advance arrival counter after the hyper workgroups' counters (chain 0's workspace)
  a.adv_cnt = advance && sd.ws ? reinterpret_cast<unsigned*>(sd.ws + pl.hpl_off + pl.n_rt_pad +
                                                              DGPRF_MAX_LAYERS)
                               : nullptr;
  a.step_adv = const_cast<int64_t*>(sd.step);
  if (advance && !a.adv_cnt) return hipErrorInvalidValue;
  a.B = pl.batch;
  a.d_in = pl.d_in;
  a.yb_cols = pl.yb_cols;
  a.bd = sd.bd;
  a.xb = sd.ws ? sd.ws + pl.xb_off : nullptr;
  a.yb = sd.ws ? sd.ws + pl.yb_off : nullptr;
  const int64_t quads = ((int64_t)a.e_end + 3) / 4;
  a.upd_blocks = (int)((quads + UPD_THREADS - 1) / UPD_THREADS);
  const bool gin = grad_in != nullptr, gonly = ud.grad_only != 0;
  const bool fb = sd.full_bayes && !gin;
  // full_bayesian=True: hyper workgroups first (per layer ceil(d R / HYP_EPB) for the Omega
  // rebuild, one in gradient-only mode), then the lik_log_var workgroup
  a.hyp_blocks = 0;
  a.pad_h = 0;
  std::memset(&a.hk, 0, sizeof(a.hk));
  size_t lds = 0;
  if (fb) {
    HypK& k = a.hk;
    k.hyp = sd.hyp;
    k.hmom = sd.hmom;
    k.hmass = sd.hmass;
    k.z = sd.z;
    k.omega = sd.omega;
    k.der = sd.der;
    k.ws = sd.ws;
    k.hyp_cs = sd.hyp_cs;
    k.om_cs = sd.om_cs;
    k.der_cs = sd.der_cs;
    k.hyp_total = pl.hyp_total;
    k.cnt_off = pl.hpl_off + pl.n_rt_pad;
    k.flags = pl.hyp_flags;
    k.likelihood = pl.likelihood;
    int nb_total = 0, hsmax = 4;
    for (int l = 0; l < pl.n_layers; ++l) {
      const int64_t n_el = (int64_t)pl.d[l] * pl.n_rf[l];
      const int nb = gonly ? 1 : (int)((n_el + HYP_EPB - 1) / HYP_EPB);
      k.d[l] = pl.d[l];
      k.R[l] = pl.n_rf[l];
      k.kind[l] = pl.kind[l];
      k.ard[l] = pl.ard[l];
      k.ns[l] = pl.ns[l];
      k.nb[l] = nb < 1 ? 1 : nb;
      k.b0[l] = nb_total;
      nb_total += k.nb[l];
      k.lis_off[l] = pl.lis_off[l];
      k.mean_off[l] = pl.mean_off[l];
      k.om_off[l] = pl.omega_off[l];
      k.hpp_off[l] = pl.hpp_off[l];
      hsmax = max(hsmax, round4(2 * pl.d[l] + 1));
      if (n_el >= (int64_t)1 << 29 || (int64_t)pl.n_rt_pad * NSM * round4(2 * pl.d[l] + 1) >= (int64_t)1 << 29)
        return hipErrorInvalidValue;  // 32-bit buffer offsets
    }
    k.hpl_off = pl.hpl_off;
    k.n_blocks = nb_total + 1;
    a.hyp_blocks = k.n_blocks;
    lds = (size_t)(5 * hsmax + max(4 * UPD_THREADS, hsmax) + UPD_THREADS + 4) * sizeof(float);
  }
  const int64_t gblocks = !a.gather_next ? 0 : (pl.d_in > GATHER_WIDE ? pl.batch
                                                    : (pl.batch + UPD_THREADS - 1) / UPD_THREADS);
  a.gather_blocks = (int32_t)gblocks;
  // resident A_1 rows of step t+1 (one-wave blocks, one per row and 1,024-float part)
  a.a1_parts = (pl.n_rf[0] + A1_PART - 1) / A1_PART;
  a.a0 = sd.ws && pl.a0_off >= 0 ? sd.ws + pl.a0_off : nullptr;
  const int64_t ablocks = a.gather_next && sd.bd.A1 && a.a0 ? (int64_t)pl.batch * a.a1_parts : 0;
  const int64_t blocks = a.hyp_blocks + a.upd_blocks + gblocks + ablocks;
  dim3 grid((unsigned)blocks, pl.n_chains);
  const bool xi = ud.xi != nullptr || ud.xi_resample != nullptr ||
                  (fb && (ud.xi_hyp != nullptr || ud.xi_hyp_resample != nullptr));
  const bool cyc = ud.schedule == DGPRF_SCHED_CYCLICAL;
  const int sel = (gin ? 8 : 0) | (gonly ? 4 : 0) | (xi ? 2 : 0) | (cyc ? 1 : 0);
#define DGPRF_UPD_CASE(S)                                                                     \
  case S:                                                                                    \
    if (lds > 65536)                                                                         \
      dgprf::set_lds_limit(                                                                  \
          (const void*)k_step_update<(S & 8) != 0, (S & 4) != 0, (S & 2) != 0, (S & 1) != 0>, lds); \
    hipLaunchKernelGGL((k_step_update<(S & 8) != 0, (S & 4) != 0, (S & 2) != 0, (S & 1) != 0>), \
                       grid, dim3(UPD_THREADS), lds, s, a);                                  \
    break;
  switch (sel) {
    DGPRF_UPD_CASE(0) DGPRF_UPD_CASE(1) DGPRF_UPD_CASE(2) DGPRF_UPD_CASE(3)
    DGPRF_UPD_CASE(4) DGPRF_UPD_CASE(5) DGPRF_UPD_CASE(6) DGPRF_UPD_CASE(7)
    DGPRF_UPD_CASE(8) DGPRF_UPD_CASE(9) DGPRF_UPD_CASE(10) DGPRF_UPD_CASE(11)
    DGPRF_UPD_CASE(12) DGPRF_UPD_CASE(13) DGPRF_UPD_CASE(14) DGPRF_UPD_CASE(15)
  }
#undef DGPRF_UPD_CASE
  return hipGetLastError();
}


hipError_t launch_agemm(const float* X, int64_t n, int ld, int d, const float* om, int R,
                        float* aout, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipError_t err = hipSuccess;
  if (n <= INT32_MAX && own_agemm(X, n, n, ld, d, om, R, aout, 1, 0, 0, 0, 1, 0, s, &err)) return err;
  if (n > INT32_MAX || (int64_t)n * ld >= ((int64_t)1 << 29) || (int64_t)d * R >= ((int64_t)1 << 29))
    return hipErrorInvalidValue;  // 32-bit buffer offsets
  AgemmK g;
  g.xrows = X;
  g.om = om;
  g.aout = aout;
  g.xrow_cs = g.om_cs = g.ws_cs = 0;
  g.B = (int32_t)n;
  g.d = d;
  g.R = R;
  g.d_in = ld;
  g.n_out = (int32_t)n;
  g.pad = 0;
  dim3 grid((unsigned)((R + 63) / 64), (unsigned)((n + 31) / 32), 1);
  hipLaunchKernelGGL(k_step_agemm, grid, dim3(256), 0, s, g);
  return hipGetLastError();
}

hipError_t launch_gather(const dgprf_plan_t& pl, const StepDev& sd, hipStream_t s) {
  if (sd.bd.mode == DGPRF_BATCH_DIRECT) return hipSuccess;
  GatherK a;
  a.bd = sd.bd;
  a.step = sd.step;
  a.xb = sd.ws + pl.xb_off;
  a.yb = sd.ws + pl.yb_off;
  a.a0 = pl.a0_off >= 0 ? sd.ws + pl.a0_off : nullptr;
  a.ws_cs = pl.ws_chain;
  a.B = pl.batch;
  a.d_in = pl.d_in;
  a.yb_cols = pl.yb_cols;
  a.step_offset = sd.step_offset;
  const int rows_per_block = pl.d_in > GATHER_WIDE ? 4 : 256;
  a.row_blocks = (pl.batch + rows_per_block - 1) / rows_per_block;
  a.a1_parts = (pl.n_rf[0] + A1_PART - 1) / A1_PART;
  // resident A_1: 4 (row, part) waves per 256-thread block
  const int ablocks = sd.bd.A1 && a.a0 ? (pl.batch * a.a1_parts + 3) / 4 : 0;
  dim3 grid((unsigned)(a.row_blocks + ablocks), pl.n_chains);
  hipLaunchKernelGGL(k_gather, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_fresh_omega(const dgprf_plan_t& pl, const StepDev& sd, hipStream_t s) {
  if (!sd.hyp) return hipErrorInvalidValue;
  const int64_t quads = (pl.omega_total + 3) / 4;
  dim3 grid((unsigned)((quads + 255) / 256), pl.n_chains);
  hipLaunchKernelGGL(k_fresh_omega, grid, dim3(256), 0, s, pl, sd.hyp, sd.ws, sd.step, sd.seed,
                     sd.step_offset, sd.omega, sd.om_cs, step_fused_fwd(pl) ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_advance(int64_t* step, int64_t by, hipStream_t s) {
  hipLaunchKernelGGL(k_advance, dim3(1), dim3(64), 0, s, step, by);
  return hipGetLastError();
}

}  // namespace dgprf
