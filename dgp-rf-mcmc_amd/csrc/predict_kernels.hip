// predict_kernels.hip — forward / predictive scoring of posterior samples on gfx950.
//
// k_forward_rows replaces, for one posterior sample theta_s (or C chains at once):
//   BNN_from_list(_input_cat).__call__      utils.py:10-16, 32-44
//   RegressionDGP.eval_log_likelihood_and_se models/regression_model.py:33-50
//   ClassificationDGP.eval_log_likelihood    models/classification_model.py:49-60
//   feed_forward_all_layers                  models/regression_model.py:24-31
// and fuses the driver's posterior-predictive log-sum-exp over samples
// (experiments/utils_training.py:79-85) as an online (max, sum) accumulator per test point.
//
// Geometry: one workgroup = one 16-row tile walking ALL layers; its 4 waves split each layer's RF
// features (16-feature chunks on v_mfma_f32_16x16x4_f32) and sum their F partials in LDS, so the
// layer outputs never leave LDS and no cross-workgroup reduction exists.
#include <algorithm>
#include <cstdlib>

#include "dgprf_internal.h"

namespace {

constexpr int NW = DGPRF_WAVES;
constexpr int ROWS16_WPE = 8;  // waves per SIMD the 16-wave row kernel is budgeted for (two per CU)
constexpr int ROWS16_CG = 1;   // 16-feature chunks per fragment-load group in the 16-wave row kernel
constexpr int TR = DGPRF_TILE_ROWS;
constexpr float LOG_2PI = 1.8378770664093453f;

__host__ __device__ __forceinline__ int round4(int x) { return (x + 3) & ~3; }

struct FwdLds {
  int xst, ftst, red_off, ft_off, total;
};

__host__ __device__ inline FwdLds fwd_lds(const dgprf_plan_t& pl, int nwr = NW, int tt = 1) {
  int dmax = 4, gmax = 1;
  for (int l = 0; l < pl.n_layers; ++l) {
    dmax = pl.d[l] > dmax ? pl.d[l] : dmax;
    gmax = pl.n_gp[l] > gmax ? pl.n_gp[l] : gmax;
  }
  FwdLds L;
  L.xst = round4(dmax) + 1;
  L.ftst = round4(gmax) + 1;
  L.red_off = round4(tt * TR * L.xst);
  // per-wave F partials [tt tiles x 16 rows][16 x output tiles + 4]: sized for the model's widest
  // layer, so the 8- and 16-wave kernels fit two workgroups per CU
  L.ft_off = L.red_off + nwr * tt * TR * ((((gmax + 15) >> 4) << 4) + 4);
  L.total = L.ft_off + round4(tt * TR * L.ftst);
  return L;
}

struct FOut {
  float* p[DGPRF_MAX_LAYERS];
};

// One wave's F partial of one layer over its features (chunks wave, wave + NWR, ...), written to
// red[wave][16][NOT*16 + 4].  Chunks go in groups of CG (4 for 4-wave tiles with NOT == 1, else 2): the group's Omega / W
// fragments are loaded together (one L2 round trip per group instead of per chunk) and its chunks'
// MFMA chains are independent; cos and sin products accumulate in separate chains.  G1 (g == 1):
// the W^T Phi^T product is a per-lane dot product (VALU) reduced over the 4 lane groups, instead of
// a 16x16 MFMA tile that would be 15/16 padding.
// NKS: k-steps of A = Omega^T x when SMALLD (2, 3, 4 or 8 >= ceil(d / 4), picked per layer by the
// caller): compile-time, so the Omega loads and A-tile MFMAs carry no per-k-step branch (a runtime
// count put every load and MFMA behind its own branch and wait: ≈2 us per chunk group on config 3);
// k-steps past d load zeros (out-of-range buffer offsets) against zero x fragments.
template <bool SMALLD, int NOT, bool RBF, bool G1, int NWR, int NKS, int TT = 1>
__device__ __forceinline__ void layer_partial(const float* __restrict__ om,
                                              const float* __restrict__ W, int R, int d, int g,
                                              float cl, const float* xs, int xst, float* red,
                                              int wave, int lr, int lq,
                                              const float* __restrict__ arow = nullptr) {
  constexpr int CG = NWR >= 16 ? ROWS16_CG : ((NWR >= 8 || NOT > 1) ? 2 : 4);
  static_assert(NKS == 2 || NKS == 3 || NKS == 4 || NKS == 8, "k-step bucket");
  // TT tiles per workgroup (rows t * 16 + lr): every Omega / W fragment serves all of them
  static_assert(TT == 1 || SMALLD, "two-tile workgroups: register-fragment path only");
  float xf[TT][NKS];
#pragma unroll
  for (int t = 0; t < TT; ++t)
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
      xf[t][ks] = (SMALLD && 4 * ks < d) ? xs[(t * TR + lr) * xst + 4 * ks + lq] : 0.f;
  const int nks = (d + 3) >> 2;  // k-steps of the !SMALLD loop
  float omk[CG][NKS], wf[CG][NOT][4][2];
  // buffer loads: 32-bit offsets (one VGPR per address), masked lanes read 0 without traffic
  const rsrc_t ro = make_rsrc(om, SMALLD ? (int64_t)d * R : 0);
  const rsrc_t rw = make_rsrc(W, (int64_t)(RBF ? 2 : 1) * R * g);
  auto load_frag = [&](int j, int f0) {
    const int fa = f0 + lr;
    if (SMALLD) {
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const int k = 4 * ks + lq;
        omk[j][ks] = bload1(ro, fa < R && k < d ? (uint32_t)((k * R + fa) * 4) : DGPRF_OOB);
      }
    }
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot) {
      const int o = G1 ? 0 : ot * 16 + lr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int fr = f0 + 4 * lq + r;
        const bool ok = o < g && fr < R;
        wf[j][ot][r][0] = bload1(rw, ok ? (uint32_t)((fr * g + o) * 4) : DGPRF_OOB);
        wf[j][ot][r][1] = RBF ? bload1(rw, ok ? (uint32_t)(((R + fr) * g + o) * 4) : DGPRF_OOB) : 0.f;
      }
    }
  };
  f4 acc[TT][NOT], acs[TT][NOT];
  float dot[TT];
#pragma unroll
  for (int t = 0; t < TT; ++t) {
    dot[t] = 0.f;
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot) acc[t][ot] = acs[t][ot] = f4zero();
  }
  constexpr int STEP = NWR * 16;
  for (int base = wave * 16; base < R; base += CG * STEP) {
#pragma unroll
    for (int j = 0; j < CG; ++j)
      if (base + j * STEP < R) load_frag(j, base + j * STEP);
#pragma unroll
    for (int j = 0; j < CG; ++j) {
      const int f0 = base + j * STEP;
      if (f0 >= R) break;
#pragma unroll
      for (int t = 0; t < TT; ++t) {
      f4 at = f4zero();
      if (SMALLD) {
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) at = mfma16(omk[j][ks], xf[t][ks], at);
      } else if (arow) {  // precomputed A row (wide first layer): A[row lr][f0 + 4lq + r]
        at = *reinterpret_cast<const f4*>(arow + f0 + 4 * lq);
      } else {
        const int fa = f0 + lr;
        for (int ks = 0; ks < nks; ++ks) {
          const int k = 4 * ks + lq;
          const float o = (fa < R && k < d) ? om[(int64_t)k * R + fa] : 0.f;
          at = mfma16(o, xs[lr * xst + 4 * ks + lq], at);
        }
      }
      float p0[4], p1[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (RBF) {
          float sn, cs;
          rf_sincos(at[r], &sn, &cs);
          p0[r] = cl * cs;
          p1[r] = cl * sn;
        } else {
          p0[r] = cl * fmaxf(at[r], 0.f);
          p1[r] = 0.f;
        }
      }
      if (G1) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          dot[t] = fmaf(p0[r], wf[j][0][r][0], dot[t]);
          if (RBF) dot[t] = fmaf(p1[r], wf[j][0][r][1], dot[t]);
        }
      } else {
#pragma unroll
        for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            acc[t][ot] = mfma16(wf[j][ot][r][0], p0[r], acc[t][ot]);
            if (RBF) acs[t][ot] = mfma16(wf[j][ot][r][1], p1[r], acs[t][ot]);
          }
      }
      }
    }
  }
  // row stride GPS = 16 NOT + 4: conflict-free 16-byte row writes (16 NOT put every row on one bank)
  constexpr int GPS = NOT * 16 + 4;
  float* redw = red + wave * TT * TR * GPS;
#pragma unroll
  for (int t = 0; t < TT; ++t) {
    float* rt = redw + t * TR * GPS;
    if (G1) {
      float v = dot[t];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      if (lq == 0) rt[lr * GPS] = v;
    } else {
      // acc[t][ot][r] = F partial[tile t, row lr][ot*16 + 4lq + r]
#pragma unroll
      for (int ot = 0; ot < NOT; ++ot)
        *reinterpret_cast<f4*>(rt + lr * GPS + ot * 16 + 4 * lq) = acc[t][ot] + acs[t][ot];
    }
  }
}

// One sample's log p (and squared error) of row idx folded into the online log-sum-exp
// accumulators (experiments/utils_training.py:79-85): m' = max(m, lp), s' = s e^{m-m'} + e^{lp-m'}.
// The pair kernel's in-place fold and k_lse_fold_samples share it, so both give the same bits.
__device__ __forceinline__ void lse_fold1(float* __restrict__ lse_m, float* __restrict__ lse_s,
                                          float* __restrict__ se_sum, int64_t idx, float lp,
                                          float se) {
  const float m0 = lse_m[idx], s0 = lse_s[idx];
  const float m1 = fmaxf(m0, lp);
  lse_s[idx] = s0 * expf(m0 - m1) + expf(lp - m1);
  lse_m[idx] = m1;
  if (se_sum) se_sum[idx] += se;
}

// One workgroup = one 16-row tile; its NWR waves split each layer's RF features (16-feature chunks
// w, w + NWR, ...) and the per-wave F partials are summed in LDS in wave order.  NWR = 16 (4 waves
// per SIMD) for test sets too small to fill the chip with the one-wave-per-tile tile kernel.
// NWR = 8 / 16 are budgeted for two workgroups per CU (4 / 8 waves per SIMD): with one, a test set
// of more tiles than CUs (config 3: 286) runs in two rounds.
// TT = 2: two 16-row tiles per workgroup (16 waves, one workgroup per CU), every W / Omega
// fragment a wave loads serves both tiles — the choice once the tiles outnumber the CUs, where a CU
// has to run two tiles anyway and two one-tile workgroups would each fetch the whole model.
// WPE: waves per SIMD the registers are budgeted for — 8 for 16-wave workgroups that may share a
// CU (explicit DGPRF_FWD_ROWS16 past one tile per CU), 4 when each CU holds one workgroup (the
// 16-wave kernel then keeps its fragments in registers instead of spilling).
template <bool SMALLD, int NOTMAX, int NWR, int TT = 1,
          int WPE = (NWR == 16 ? ROWS16_WPE : (NWR == 8 ? 4 : 1))>
__global__ __launch_bounds__(64 * NWR)
__attribute__((amdgpu_waves_per_eu(TT > 1 ? 4 : WPE)))
void k_forward_rows(
    const dgprf_plan_t pl, const float* __restrict__ theta, const float* __restrict__ omega,
    const float* __restrict__ der, const float* __restrict__ X, const float* __restrict__ Y,
    const int y_cols, const int64_t n, const FOut fo, float* __restrict__ logp_out,
    float* __restrict__ se_out, float* __restrict__ lse_m, float* __restrict__ lse_s,
    float* __restrict__ se_sum, const float* __restrict__ a0, const int64_t row_begin,
    const int64_t row_end) {
  // rows [row_begin, row_end) of the n-row set; a0 = A_1 = X Omega_1 of those rows
  // ([row - row_begin][R_1], k_step_agemm) for a wide first layer, or nullptr
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const FwdLds LD = fwd_lds(pl, NWR, TT);
  const int chain = blockIdx.y;
  const int64_t ochain = pl.hyp_per_chain ? (int64_t)chain * pl.omega_total : 0;
  const int64_t dchain = pl.hyp_per_chain ? (int64_t)chain * pl.der_total : 0;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, lr = lane & 15, lq = lane >> 4;
  const int64_t row0 = row_begin + (int64_t)blockIdx.x * TR * TT;
  float* xs = smem;
  float* red = smem + LD.red_off;
  float* ft = smem + LD.ft_off;
  const float* Wc = theta + ((int64_t)blockIdx.z * pl.n_chains + chain) * pl.w_total;
  const int L = pl.n_layers;

  for (int layer = 0; layer < L; ++layer) {
    const int d = pl.d[layer], dpad = round4(d);
    const int R = pl.n_rf[layer], g = pl.n_gp[layer];
    const int gp = layer > 0 ? pl.n_gp[layer - 1] : 0;
    const float* arow = (layer == 0 && a0) ? a0 + (row0 - row_begin + lr) * (int64_t)R : nullptr;
    for (int e = threadIdx.x; !arow && e < TT * TR * dpad; e += blockDim.x) {
      const int r = e / dpad, k = e - r * dpad;
      const int64_t b = row0 + r;
      float v = 0.f;
      if (b < row_end && k < d) v = (k < gp) ? ft[r * LD.ftst + k] : X[b * pl.d_in + (k - gp)];
      xs[r * LD.xst + k] = v;
    }
    __syncthreads();

    {
      const float* __restrict__ om = omega + ochain + pl.omega_off[layer];
      const float* __restrict__ W = Wc + pl.w_off[layer];
      const float cl = der[dchain + layer];
      const int NOT = (g + 15) >> 4;
      const bool rbf = pl.kind[layer] == DGPRF_RBF;
      // runtime (layer) -> compile-time body: output tiles, kernel kind, g == 1 VALU path; layers
      // with d <= 32 take the register-fragment path even when another layer is wide
#define DGPRF_LP(SD, NT, RB, G1_)                                                               \
  do {                                                                                          \
    if (!SD || d > 16)                                                                          \
      layer_partial<SD, NT, RB, G1_, NWR, 8, TT>(om, W, R, d, g, cl, xs, LD.xst, red, wave, lr, lq, arow); \
    else if (d > 12)                                                                            \
      layer_partial<SD, NT, RB, G1_, NWR, 4, TT>(om, W, R, d, g, cl, xs, LD.xst, red, wave, lr, lq, arow); \
    else if (d > 8)                                                                             \
      layer_partial<SD, NT, RB, G1_, NWR, 3, TT>(om, W, R, d, g, cl, xs, LD.xst, red, wave, lr, lq, arow); \
    else                                                                                        \
      layer_partial<SD, NT, RB, G1_, NWR, 2, TT>(om, W, R, d, g, cl, xs, LD.xst, red, wave, lr, lq, arow); \
  } while (0)
#define DGPRF_LP_ALL(SD)                                                                        \
  do {                                                                                          \
    if (g == 1) {                                                                               \
      if (rbf) DGPRF_LP(SD, 1, true, true);                                                     \
      else DGPRF_LP(SD, 1, false, true);                                                        \
    } else if (NOT == 1) {                                                                      \
      if (rbf) DGPRF_LP(SD, 1, true, false);                                                    \
      else DGPRF_LP(SD, 1, false, false);                                                       \
    } else if (NOTMAX >= 2 && NOT == 2) {                                                       \
      if (rbf) DGPRF_LP(SD, (NOTMAX >= 2 ? 2 : 1), true, false);                                \
      else DGPRF_LP(SD, (NOTMAX >= 2 ? 2 : 1), false, false);                                   \
    } else if (NOTMAX >= 3 && NOT == 3) {                                                       \
      if (rbf) DGPRF_LP(SD, (NOTMAX >= 3 ? 3 : 1), true, false);                                \
      else DGPRF_LP(SD, (NOTMAX >= 3 ? 3 : 1), false, false);                                   \
    } else if (NOTMAX >= 4) {                                                                   \
      if (rbf) DGPRF_LP(SD, (NOTMAX >= 4 ? 4 : 1), true, false);                                \
      else DGPRF_LP(SD, (NOTMAX >= 4 ? 4 : 1), false, false);                                   \
    }                                                                                           \
  } while (0)
      if constexpr (TT > 1) {  // host-selected for d <= 32 models only
        DGPRF_LP_ALL(true);
      } else {
        if (SMALLD || d <= 32) DGPRF_LP_ALL(true);
        else DGPRF_LP_ALL(false);
      }
#undef DGPRF_LP_ALL
#undef DGPRF_LP
    }
    const int GPS = ((g + 15) >> 4) * 16 + 4;  // (layer_partial's padded row stride)
    __syncthreads();
    float* out = fo.p[layer] ? fo.p[layer] + (int64_t)chain * n * g : nullptr;
    for (int e = threadIdx.x; e < TT * TR * g; e += blockDim.x) {
      const int r = e / g, o = e - r * g;
      float v = red[r * GPS + o];
#pragma unroll
      for (int w = 1; w < NWR; ++w) v += red[w * TT * TR * GPS + r * GPS + o];
      ft[r * LD.ftst + o] = v;
      const int64_t b = row0 + r;
      if (out && b < row_end) out[b * g + o] = v;
    }
    __syncthreads();
  }

  // likelihood per row (threads 0..15)
  const bool want_lik = logp_out || se_out || lse_m;
  if (want_lik && threadIdx.x < TT * TR) {
    const int64_t b = row0 + threadIdx.x;
    if (b < row_end) {
      const int g = pl.n_gp[L - 1];
      const float* f = ft + threadIdx.x * LD.ftst;
      const float* y = Y + b * y_cols;
      float lp = 0.f, se = 0.f;
      if (pl.likelihood == DGPRF_LIK_GAUSSIAN) {
        const float var = der[dchain + DGPRF_MAX_LAYERS];
        const float logvar = logf(var);
        for (int o = 0; o < g; ++o) {
          const float diff = y[o] - f[o];
          lp += -0.5f * (LOG_2PI + logvar + diff * diff / var);
          se += diff * diff;
        }
        se = se / (float)g;  // reduce_mean over outputs (regression_model.py:46)
      } else {
        float mx = -INFINITY;
        for (int o = 0; o < g; ++o) mx = fmaxf(mx, f[o]);
        float s = 0.f;
        for (int o = 0; o < g; ++o) s += expf(f[o] - mx);
        // int32(Y[:, 0]) (likelihoods/softmax.py:14); a label outside [0, g) scores NaN (TF raises)
        const int lab = (int)y[0];
        const bool lab_ok = lab >= 0 && lab < g;
        lp = lab_ok ? f[lab] - (mx + logf(s)) : __builtin_nanf("");
      }
      const int64_t idx = (int64_t)chain * n + b;
      // blockIdx.z = sample of a multi-sample launch: its outputs [sample][chain][n]
      const int64_t oidx = (int64_t)blockIdx.z * pl.n_chains * n + idx;
      if (logp_out) logp_out[oidx] = lp;
      if (se_out) se_out[oidx] = se;
      if (lse_m) lse_fold1(lse_m, lse_s, se_sum, idx, lp, se);
    }
  }
}

// Combine per-part (chain x rank) accumulators and reduce to the two scalars in a fixed order.
__global__ __launch_bounds__(1024) void k_lse_finalize(const float* __restrict__ lse_m,
                                                       const float* __restrict__ lse_s,
                                                       const float* __restrict__ se_sum,
                                                       const int parts, const int64_t n,
                                                       const double s_total, const float log_y_std,
                                                       const float y_std, float* lse_out,
                                                       double* out) {
  __shared__ double r0[1024], r1[1024];
  double a0 = 0.0, a1 = 0.0;
  const double log_s = log(s_total);
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    float m = -INFINITY;
    for (int p = 0; p < parts; ++p) m = fmaxf(m, lse_m[(int64_t)p * n + i]);
    float s = 0.f, e = 0.f;
    for (int p = 0; p < parts; ++p) {
      s += lse_s[(int64_t)p * n + i] * expf(lse_m[(int64_t)p * n + i] - m);
      if (se_sum) e += se_sum[(int64_t)p * n + i];
    }
    const float lse = m + logf(s);
    if (lse_out) lse_out[i] = lse;
    a0 += (double)lse - log_s;
    a1 += (double)e;
  }
  r0[threadIdx.x] = a0;
  r1[threadIdx.x] = a1;
  __syncthreads();
  for (int w = blockDim.x / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      r0[threadIdx.x] += r0[threadIdx.x + w];
      r1[threadIdx.x] += r1[threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[0] = r0[0] / (double)n - (double)log_y_std;
    out[1] = sqrt(r1[0] / (s_total * (double)n)) * (double)y_std;
  }
}

// Phi = c [cos(X Omega) | sin(X Omega)]  or  c relu(X Omega)  (layers/rf_layers.py:42-44,88-90)
__global__ __launch_bounds__(256) void k_rf_features(const int kind, const float* __restrict__ X,
                                                     const int64_t n, const int d,
                                                     const float* __restrict__ om, const int R,
                                                     const float* __restrict__ cptr,
                                                     float* __restrict__ phi) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, lr = lane & 15, lq = lane >> 4;
  const int64_t row0 = (int64_t)blockIdx.x * TR;
  const int f0 = (blockIdx.y * NW + wave) * 16;
  if (f0 >= R) return;
  const int P = kind == DGPRF_RBF ? 2 * R : R;
  const float cl = *cptr;
  const int fa = f0 + lr;
  const int64_t bx = row0 + lr;
  f4 at = f4zero();
  for (int k0 = 0; k0 < d; k0 += 4) {
    const int k = k0 + lq;
    const float o = (fa < R && k < d) ? om[(int64_t)k * R + fa] : 0.f;
    const float x = (bx < n && k < d) ? X[bx * d + k] : 0.f;
    at = mfma16(o, x, at);
  }
  if (bx >= n) return;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int f = f0 + 4 * lq + r;
    if (f < R) {
      if (kind == DGPRF_RBF) {
        float s, c;
        rf_sincos(at[r], &s, &c);
        phi[bx * P + f] = cl * c;
        phi[bx * P + R + f] = cl * s;
      } else {
        phi[bx * P + f] = cl * fmaxf(at[r], 0.f);
      }
    }
  }
}

// F = Phi W (layers/GP_weight_layers.py:11-15, the stand-alone GPLayer.__call__) on MFMA: a
// 256-thread workgroup owns a 16-row x 16-output tile of F; its 4 waves split K = P into 16-wide
// blocks (wave w takes blocks w, w + 4, ...), each block four v_mfma_f32_16x16x4_f32 with lane
// (lr, lq) holding Phi[row lr][k0 + 4lq .. +3] as one 16-byte load and W[k0 + 4lq + s][o lr];
// the four K-partial tiles are summed in LDS in wave order (deterministic).  Rows >= n, k >= P
// and outputs >= g read 0 through the buffer descriptors (no traffic) and are never stored.
__global__ __launch_bounds__(256) void k_gp_matmul(const float* __restrict__ phi, const int64_t n,
                                                   const int P, const float* __restrict__ W,
                                                   const int g, float* __restrict__ F) {
  __shared__ __attribute__((aligned(16))) float red[4][16][17];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, lr = lane & 15, lq = lane >> 4;
  const int64_t row0 = (int64_t)blockIdx.x * 16;
  const int o0 = (int)blockIdx.y * 16;
  const int64_t rows = min((int64_t)16, n - row0);
  const rsrc_t rp = make_rsrc(phi + row0 * P, rows * P);
  const rsrc_t rw = make_rsrc(W, (int64_t)P * g);
  const bool rok = lr < rows, ook = o0 + lr < g;
  const bool vec = (P & 3) == 0;  // 16-byte aligned Phi rows
  f4 acc = f4zero();
  const int nkb = (P + 15) >> 4;
  for (int kb = wave; kb < nkb; kb += 4) {
    const int k = kb * 16 + 4 * lq;
    f4 a;
    if (vec) {
      a = bload4(rp, rok && k < P ? (uint32_t)(((int64_t)lr * P + k) * 4) : DGPRF_OOB);
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s)
        a[s] = bload1(rp, rok && k + s < P ? (uint32_t)(((int64_t)lr * P + k + s) * 4) : DGPRF_OOB);
    }
    float b[4];
#pragma unroll
    for (int s = 0; s < 4; ++s)
      b[s] = bload1(rw, ook && k + s < P ? (uint32_t)(((int64_t)(k + s) * g + o0 + lr) * 4) : DGPRF_OOB);
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = mfma16(a[s], b[s], acc);
  }
  // acc[r] = partial F[row0 + 4lq + r][o0 + lr]
#pragma unroll
  for (int r = 0; r < 4; ++r) red[wave][4 * lq + r][lr] = acc[r];
  __syncthreads();
  const int i = threadIdx.x >> 4, j = threadIdx.x & 15;
  if (i < rows && o0 + j < g)
    F[(row0 + i) * g + o0 + j] = ((red[0][i][j] + red[1][i][j]) + red[2][i][j]) + red[3][i][j];
}

// sum_l sum log N(W_l; 0, 1) per chain (models/dgp.py:129-136), fixed-order tree reduction.
__global__ __launch_bounds__(256) void k_prior_w(const dgprf_plan_t pl,
                                                 const float* __restrict__ theta, float* out) {
  __shared__ float red[256];
  const int chain = blockIdx.x;
  const float* th = theta + (int64_t)chain * pl.w_total;
  float total = 0.f;
  for (int l = 0; l < pl.n_layers; ++l) {
    const int64_t cnt = (int64_t)pl.P[l] * pl.n_gp[l];
    float a = 0.f;
    for (int64_t i = threadIdx.x; i < cnt; i += blockDim.x) {
      const float w = th[pl.w_off[l] + i];
      a += -0.5f * (LOG_2PI + 0.f + w * w);
    }
    red[threadIdx.x] = a;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
      if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
      __syncthreads();
    }
    total += red[0];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[chain] = total;
}


// ============================================================================ tile kernel
// k_forward_tiles: the same computation as k_forward_rows for models whose layers all have
// d <= 32, g <= 64 and R % 4 == 0 (every configuration of BASELINE.json).
//   * a workgroup covers 64 rows: each wave owns a 16-row tile through ALL layers, so F accumulates
//     in the wave's registers over the whole feature loop — no cross-wave reduction;
//   * the 4 waves walk the same 64-feature blocks: each block's Omega rows (d x 64) and W rows
//     (2 x 64 x g) are fetched once per workgroup with buffer_load_dwordx4 into a double-buffered
//     LDS ring (the next block's loads are in flight while the current block computes), one barrier
//     per block;
//   * the layer output F (16 x g per wave) stays in the wave's LDS tile and is the next layer's
//     input; dataset columns ([F | X], utils.py:42) come from the wave's X rows, loaded once.
// waves per workgroup (4 waves = 4 SIMDs).  16 (one workgroup per CU) makes the per-block barrier
// keep the 4 waves of each SIMD in step — otherwise oldest-first issue arbitration starves the
// younger waves and the last ones finish alone — but measured no faster at N_t = 1e5 (lockstep
// phases overlap MFMA and VALU worse, and 1.5 rounds of 16-tile workgroups leave half the CUs idle
// in the second); DESIGN.md §4.
constexpr int TWW = 4;
constexpr int TW_THREADS = 64 * TWW;
constexpr int TW_ROWS = TWW * TR;  // rows per workgroup
constexpr int TILE_WAVES = 4;       // waves per SIMD the register budget must allow (latency hiding)
constexpr int TILE_TPW_DEFAULT = 1; // 16-row tiles per wave (2: two chains per wave, but 186 VGPRs ->
                                    // 2 waves/SIMD, slower)
constexpr bool TILE_APHASE = true;  // issue a block's four A-tile chains before its trig / F work
constexpr int TILE_LEAN_WAVES = 5;  // waves per SIMD of the lean instance (NOTMAX = 0, every layer
                                    // g, d <= 8); it computes each chunk's A tile just before use
                                    // (the A-phase there measured slower: 225 vs 213 us)
constexpr int TW_OST = 80;        // LDS row stride of a staged Omega block (conflict-free reads)
__host__ __device__ constexpr int tw_wst(int notm) { return 16 * notm + 4; }  // W row stride

struct TileLds {
  int obuf, wbuf, o_off, w_off, xin_off, xin_st, f_off, ftst, total;
  int orows;  // Omega rows staged per block (16 njo; 8 in the pair kernel, whose layers have d <= 8)
};

// the pair kernel's layer-0 W rows: [half][feature][s * 8 + o], row stride PST = 16.  (A stride of
// 20 puts lanes 16-31 of a read 16 banks away from lanes 0-15, but the ring then pushes the
// workgroup past 32 KiB of LDS: 4 workgroups per CU instead of the 5 its registers allow.)
constexpr int PST = 16;

__host__ __device__ inline TileLds tile_lds(const dgprf_plan_t& pl, int notmax, int njo, int tpw,
                                            bool wide0 = false, int spw = 1) {
  int gmax = 1;
  for (int l = 0; l < pl.n_layers; ++l) gmax = pl.n_gp[l] > gmax ? pl.n_gp[l] : gmax;
  TileLds T;
  // njo float4 per thread: 16 Omega rows each; the pair kernel (every layer d <= 8, two k-steps)
  // stages the 8 rows its k-steps read, so five of its workgroups fit a CU's 160 KiB with room
  T.orows = spw == 2 ? 8 : 16 * njo;
  T.obuf = T.orows * TW_OST;
  // [cos|sin][64 features][16 NOT + 4]; notmax = 0 (the lean instance: every layer g <= 8, d <= 8)
  // [cos|sin][64 features][8] (G8) or [cos|sin][64] (g == 1)
  T.wbuf = notmax == 0 ? (spw == 2 ? 2 * 64 * PST : 2 * 64 * 8) : 2 * 64 * tw_wst(notmax);
  T.o_off = 0;
  T.w_off = 2 * T.obuf;
  T.xin_st = wide0 ? 4 : round4(pl.d_in);  // wide0: layer 0 reads A_1, no input rows staged
  T.xin_off = T.w_off + 2 * T.wbuf;
  T.ftst = spw == 2 ? gmax : gmax + 1;  // the pair layout: 5 workgroups' LDS in 160 KiB
  T.f_off = T.xin_off + TWW * tpw * TR * T.xin_st;
  T.total = T.f_off + TWW * spw * round4(tpw * TR * T.ftst);  // spw samples' F per wave
  return T;
}

// One layer for the calling wave's 16 rows.
//   JW / JO: float4 W / Omega loads per thread per 64-feature block (16 JO Omega rows staged);
//   KS: k-steps of A = Omega^T x (ceil(d/4) <= KS <= 4 JO; extra k-steps multiply staged zeros).
// Staged layouts: Omega [k][TW_OST] (x 1/2pi for the hardware sin/cos), W [h][feature][WST] with
// WST = 16 NOT + 4 (g == 1: raw [h][64]); feature rows >= R are zeroed while staging, and output
// columns o >= g are never stored, so the fragment reads need neither masks nor clamps and all
// their offsets are immediates.
// OPQ: the lane index re-read behind an empty asm, so this layer's per-lane LDS offsets are computed
// here and not hoisted above the caller's layer loop (where, live through every layer, they pushed
// the lean instance past its 96-VGPR budget into scratch)
template <int NOT, bool RBF, bool G1, bool G8, int JW, int JO, int KS, int TPW, bool AP = true,
          bool OPQ = false>
__device__ __forceinline__ void tile_layer(const dgprf_plan_t& pl, int layer,
                                           const float* __restrict__ W,
                                           const float* __restrict__ om, float cl,
                                           const TileLds& T, float* smem, float* xin, float* ftw,
                                           int lr, int lq, int64_t wrow0, int64_t n, float* fout,
                                           const float* __restrict__ arow0 = nullptr) {
  if (OPQ) {
    int ln = (int)threadIdx.x & 63;
    asm volatile("" : "+v"(ln));
    lr = ln & 15;
    lq = ln >> 4;
  }
  // arow0 (wide first layer): A_1 rows of this wave's tiles, [row][R] (k_step_agemm); the Omega
  // staging and A-tile MFMAs are skipped and A is read straight into the accumulator layout
  // G8 (2 <= g <= 8): W rows of 8 with the columns interleaved as 2 (o & 3) + (o >> 2), so a lane's
  // two 4x4-block operands (o = i, 4 + i) are one ds_read_b64
  constexpr int WST = G8 ? 8 : tw_wst(NOT);
  constexpr bool REV = RBF && !DGPRF_PRECISE_TRIG_ON;
  constexpr bool APHASE = AP && TILE_APHASE && KS <= 2;
  // the k-steps read Omega rows 0..4KS-1 of the staged block: all of them must be staged (rows >= d
  // as zeros) — LDS is not cleared between kernels, and 0 * stale NaN is NaN
  static_assert(4 * KS <= 16 * JO, "k-steps beyond the staged Omega rows");
  const int d = pl.d[layer], R = pl.n_rf[layer], g = pl.n_gp[layer];
  const int gp = layer > 0 ? pl.n_gp[layer - 1] : 0;
  int tid = threadIdx.x;
  if (OPQ) asm volatile("" : "+v"(tid));
  const int gmag = (1048576 + g - 1) / g;  // floor(e / g) = (e * gmag) >> 20 for e < 4096
  // x fragments of the A = Omega^T x contraction: xf[t][ks] = X_l[tile t, row lr][4ks + lq]
  float xf[TPW][KS];
#pragma unroll
  for (int t = 0; t < TPW; ++t)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int col = 4 * ks + lq, row = t * TR + lr;
      const float a = ftw[row * T.ftst + min(col, T.ftst - 1)];
      const float b = xin[row * T.xin_st + min(max(col - gp, 0), T.xin_st - 1)];
      xf[t][ks] = col < gp ? a : (col < d ? b : 0.f);
    }
  const rsrc_t rw = make_rsrc(W, (int64_t)(RBF ? 2 : 1) * R * g);
  const rsrc_t ro = make_rsrc(om, (int64_t)d * R);
  const int nwq = (RBF ? 32 : 16) * g;  // float4 of one W block
  f4 sw[JW], so[JO];
  const bool stager = tid < 256;  // the staging counts JW / JO are per 256 threads
  auto stage_load = [&](int fb) {
    if (!stager) return;
#pragma unroll
    for (int j = 0; j < JW; ++j) {
      const int i = tid + 256 * j, h = i >= 16 * g, q = i - h * 16 * g;
      sw[j] = bload4(rw, i < nwq ? (uint32_t)((((h * R) + fb) * g + 4 * q) * 4) : DGPRF_OOB);
    }
#pragma unroll
    for (int j = 0; j < JO; ++j) {
      const int i = tid + 256 * j, k = i >> 4, c4 = i & 15;
      so[j] = bload4(ro, !arow0 && k < d && fb + 4 * c4 < R ? (uint32_t)((k * R + fb + 4 * c4) * 4)
                                                           : DGPRF_OOB);
    }
  };
  auto stage_store = [&](int buf, int fb) {
    if (!stager) return;
    float* wsb = smem + T.w_off + buf * T.wbuf;
    float* osb = smem + T.o_off + buf * T.obuf;
#pragma unroll
    for (int j = 0; j < JW; ++j) {
      const int i = tid + 256 * j;
      if (i < nwq) {
        const int h = i >= 16 * g, e0 = 4 * (i - h * 16 * g);
        if (G1) {  // raw [h][64]: rows e0..e0+3
          f4 v = sw[j];
#pragma unroll
          for (int t = 0; t < 4; ++t) v[t] = fb + e0 + t < R ? v[t] : 0.f;
          *reinterpret_cast<f4*>(wsb + h * 64 + e0) = v;
        } else if (G8) {
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const int e = e0 + t, row = (e * gmag) >> 20, col = e - row * g;
            if (row < 64)
              wsb[(h * 64 + row) * WST + 2 * (col & 3) + (col >> 2)] = fb + row < R ? sw[j][t] : 0.f;
          }
        } else if ((g & 3) == 0) {  // the float4 lies in one row
          const int row = (e0 * gmag) >> 20, col = e0 - row * g;
          const f4 v = fb + row < R ? sw[j] : f4zero();
          *reinterpret_cast<f4*>(wsb + (h * 64 + row) * WST + col) = v;
        } else {
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const int e = e0 + t, row = (e * gmag) >> 20, col = e - row * g;
            if (row < 64) wsb[(h * 64 + row) * WST + col] = fb + row < R ? sw[j][t] : 0.f;
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < JO; ++j) {
      const int i = tid + 256 * j;
      if ((i >> 4) < T.orows)
        *reinterpret_cast<f4*>(osb + (i >> 4) * TW_OST + 4 * (i & 15)) =
            REV ? so[j] * 0.15915494309189535f : so[j];
    }
  };

  f4 acc[TPW][NOT], acs[TPW][NOT];
  // G8: 4x4-block accumulators [t][h]: lane (lq, lr) reg i = F[row lr][4h + i] over features 4lq..
  f4 a8[TPW][2], s8[TPW][2];
  float dot[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    dot[t] = 0.f;
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot) acc[t][ot] = acs[t][ot] = f4zero();
    a8[t][0] = a8[t][1] = s8[t][0] = s8[t][1] = f4zero();
  }
  const int nb = (R + 63) >> 6;
  stage_load(0);
  stage_store(0, 0);
  __syncthreads();
  for (int blk = 0; blk < nb; ++blk) {
    const int fb = blk * 64, buf = blk & 1;
    if (blk + 1 < nb) stage_load(fb + 64);
    const float* wsb = smem + T.w_off + buf * T.wbuf;
    const float* osb = smem + T.o_off + buf * T.obuf + lq * TW_OST + lr;
    const float* wl = wsb + (G1 ? 4 * lq : (G8 ? 4 * lq * WST + 2 * (lr & 3) : 4 * lq * WST + lr));
    // A[tile t, row lr][feature fb + 16c + 4lq + r]; the Omega / W fragments serve every tile.
    // APHASE: the four chunks' A tiles are issued together first (independent MFMA chains, so their
    // dependent latency overlaps), and the trig + F contraction of chunk c follows.
    f4 atc[APHASE ? 4 : 1][TPW];
    if (APHASE && !arow0) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float om[KS];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) om[ks] = osb[4 * ks * TW_OST + 16 * c];
#pragma unroll
        for (int t = 0; t < TPW; ++t) {
          atc[c][t] = f4zero();
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) atc[c][t] = mfma16(om[ks], xf[t][ks], atc[c][t]);
        }
      }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      f4 at[TPW];
      if (arow0) {
        // A_1 is in radians; the staged-Omega path computes it in revolutions (Omega x 1/2pi)
#pragma unroll
        for (int t = 0; t < TPW; ++t) {
          at[t] = *reinterpret_cast<const f4*>(arow0 + (int64_t)(t * TR + lr) * R + fb + 16 * c + 4 * lq);
          if (REV) at[t] = at[t] * 0.15915494309189535f;
        }
      } else if (APHASE) {
#pragma unroll
        for (int t = 0; t < TPW; ++t) at[t] = atc[c][t];
      } else {
        float om[KS];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) om[ks] = osb[4 * ks * TW_OST + 16 * c];
#pragma unroll
        for (int t = 0; t < TPW; ++t) {
          at[t] = f4zero();
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) at[t] = mfma16(om[ks], xf[t][ks], at[t]);
        }
      }
      // features without the scale c (applied once to F): cos/sin(A) or relu(A)
      float p0[TPW][4], p1[TPW][4];
#pragma unroll
      for (int t = 0; t < TPW; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (REV) {
            const float u = __builtin_amdgcn_fractf(at[t][r]);
            p0[t][r] = __builtin_amdgcn_cosf(u);
            p1[t][r] = __builtin_amdgcn_sinf(u);
          } else if (RBF) {
            float sv, cv;
            rf_sincos(at[t][r], &sv, &cv);
            p0[t][r] = cv;
            p1[t][r] = sv;
          } else {
            p0[t][r] = fmaxf(at[t][r], 0.f);
            p1[t][r] = 0.f;
          }
        }
      if (G1) {
        const f4 w0 = *reinterpret_cast<const f4*>(wl + 16 * c);
        const f4 w1 = RBF ? *reinterpret_cast<const f4*>(wl + 64 + 16 * c) : f4zero();
#pragma unroll
        for (int t = 0; t < TPW; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            dot[t] = fmaf(p0[t][r], w0[r], dot[t]);
            if (RBF) dot[t] = fmaf(p1[t][r], w1[r], dot[t]);
          }
      } else if (G8) {
        // 4x4x1 blocks: block b = 4 lq + (lr >> 2) covers rows 4 (b & 3) + j and feature 4 lq + r;
        // A = W[feature][4h + (lr & 3)], B = this lane's cos / sin value.  (The cos half on 16x16x4
        // tiles instead measured slower: 241 vs 221 us per config-2 sample.)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          typedef float f2v __attribute__((ext_vector_type(2)));
          const f2v wc = *reinterpret_cast<const f2v*>(wl + (16 * c + r) * WST);
          f2v wsn = {0.f, 0.f};
          if (RBF) wsn = *reinterpret_cast<const f2v*>(wl + (64 + 16 * c + r) * WST);
#pragma unroll
          for (int t = 0; t < TPW; ++t) {
            a8[t][0] = mfma4(wc[0], p0[t][r], a8[t][0]);
            a8[t][1] = mfma4(wc[1], p0[t][r], a8[t][1]);
            if (RBF) {
              s8[t][0] = mfma4(wsn[0], p1[t][r], s8[t][0]);
              s8[t][1] = mfma4(wsn[1], p1[t][r], s8[t][1]);
            }
          }
        }
      } else {
#pragma unroll
        for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int off = (16 * c + r) * WST + 16 * ot;
            const float w0 = wl[off];
            const float w1 = RBF ? wl[64 * WST + off] : 0.f;
#pragma unroll
            for (int t = 0; t < TPW; ++t) {
              acc[t][ot] = mfma16(w0, p0[t][r], acc[t][ot]);
              if (RBF) acs[t][ot] = mfma16(w1, p1[t][r], acs[t][ot]);
            }
          }
      }
    }
    if (blk + 1 < nb) stage_store(buf ^ 1, fb + 64);
    __syncthreads();
  }
  // F tiles of this wave -> ftw (the next layer's input) and the optional per-layer output
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    const int row = t * TR + lr;
    const int64_t b = wrow0 + row;
    if (G1) {
      float v = dot[t];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      v *= cl;
      if (lq == 0) {
        ftw[row * T.ftst] = v;
        if (fout && b < n) fout[b] = v;
      }
    } else if (G8) {
      // sum the four feature groups (lanes lr, lr + 16, lr + 32, lr + 48)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float v = a8[t][h][i] + s8[t][h][i];
          v += __shfl_xor(v, 16);
          v += __shfl_xor(v, 32);
          const int o = 4 * h + i;
          if (lq == 0 && o < g) {
            v *= cl;
            ftw[row * T.ftst + o] = v;
            if (fout && b < n) fout[b * g + o] = v;
          }
        }
    } else {
      // acc[t][ot][r] = F[tile t, row lr][ot*16 + 4lq + r] / c
#pragma unroll
      for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int o = ot * 16 + 4 * lq + r;
          if (o < g) {
            const float v = cl * (acc[t][ot][r] + acs[t][ot][r]);
            ftw[row * T.ftst + o] = v;
            if (fout && b < n) fout[b * g + o] = v;
          }
        }
    }
  }
  __syncthreads();  // ftw complete before the next layer reads its x fragments
}

// Layer 0 of TWO posterior samples at once (pair kernel, lean models: every layer d, g <= 8).
// Omega_1 and the layer input are the same for every sample — z is drawn once at construction
// (layers/rf_layers.py:21-22) and the samples differ only in W — so A = X Omega_1 (:42-44) and its
// cos / sin (or relu) are computed once for both.  The F contraction then has 2 g_0 <= 16 real
// output columns and runs on v_mfma_f32_16x16x4_f32: A operand = [W_s0 | W_s1]^T (output column
// i = 8 s + o), B = Phi^T; the 16x16x4 MFMA holds the SIMD issue port for 8 of its 32 cycles where
// the 4x4x1 blocks of the one-sample body hold it for all of theirs (MI355X_MICROARCH.md).  Both
// samples' W blocks are staged per 64-feature block in a double-buffered LDS ring with the Omega
// block; columns o >= g_0 of a sample's eight stay whatever the ring held: they only feed output
// rows that are never stored.  F_s (scaled by c_1) goes to the wave's F tile of sample s.
template <bool RBF>
__device__ __forceinline__ void tile_layer0_pair(const dgprf_plan_t& pl, const float* __restrict__ W0,
                                                 const float* __restrict__ W1,
                                                 const float* __restrict__ om, float cl,
                                                 const TileLds& T, float* smem, const float* xin,
                                                 float* ftw0, float* ftw1, int lr, int lq) {
  constexpr int KS = 2;
  constexpr bool REV = RBF && !DGPRF_PRECISE_TRIG_ON;
  const int d = pl.d[0], R = pl.n_rf[0], g = pl.n_gp[0];
  // lane / thread index behind an empty asm (as tile_layer's OPQ): this layer's per-lane offsets
  // are computed here, not hoisted into registers live through the later layers
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  lr = tid & 15;
  lq = (tid & 63) >> 4;
  const int gmag = (1048576 + g - 1) / g;  // floor(e / g) = (e * gmag) >> 20 for e < 4096
  float xf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int col = 4 * ks + lq;
    xf[ks] = col < d ? xin[lr * T.xin_st + min(col, T.xin_st - 1)] : 0.f;
  }
  // one descriptor over both samples' W (W1 - W0 is uniform: C w_total floats, or 0 for an odd
  // last sample), so no load picks its descriptor per lane
  const int64_t wn = (int64_t)(RBF ? 2 : 1) * R * g, sd1 = (int64_t)(W1 - W0);
  const rsrc_t rw = make_rsrc(W0, sd1 + wn);
  const rsrc_t ro = make_rsrc(om, (int64_t)d * R);
  const int nh4 = 16 * g;  // float4 of one half's 64-feature block
  f4 sw[2], so;
  auto stage_load = [&](int fb) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {  // i < 2 samples x (RBF ? 2 : 1) halves x 16 g
      const int i = tid + 256 * j, sidx = i >= 2 * nh4, q = i - sidx * 2 * nh4, h = q >= nh4;
      const int e4 = q - h * nh4;
      const bool ok = (RBF || h == 0) && i < 4 * nh4;
      const uint32_t off = (uint32_t)((sidx * sd1 + ((h * R) + fb) * g + 4 * e4) * 4);
      sw[j] = bload4(rw, ok ? off : DGPRF_OOB);
    }
    const int k = tid >> 4, c4 = tid & 15;
    so = bload4(ro, k < d && fb + 4 * c4 < R ? (uint32_t)((k * R + fb + 4 * c4) * 4) : DGPRF_OOB);
  };
  auto stage_store = [&](int buf, int fb) {
    float* wsb = smem + T.w_off + buf * T.wbuf;
    float* osb = smem + T.o_off + buf * T.obuf;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int i = tid + 256 * j, sidx = i >= 2 * nh4, q = i - sidx * 2 * nh4, h = q >= nh4;
      const int e0 = 4 * (q - h * nh4);
      if ((RBF || h == 0) && i < 4 * nh4) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int e = e0 + t, row = (e * gmag) >> 20, col = e - row * g;
          if (row < 64) wsb[(h * 64 + row) * PST + 8 * sidx + col] = fb + row < R ? sw[j][t] : 0.f;
        }
      }
    }
    if ((tid >> 4) < T.orows)
      *reinterpret_cast<f4*>(osb + (tid >> 4) * TW_OST + 4 * (tid & 15)) =
          REV ? so * 0.15915494309189535f : so;
  };
  f4 acc = f4zero(), acs = f4zero();
  const int nb = (R + 63) >> 6;
  stage_load(0);
  stage_store(0, 0);
  __syncthreads();
  for (int blk = 0; blk < nb; ++blk) {
    const int fb = blk * 64, buf = blk & 1;
    if (blk + 1 < nb) stage_load(fb + 64);
    const float* wl = smem + T.w_off + buf * T.wbuf + 4 * lq * PST + lr;
    const float* osb = smem + T.o_off + buf * T.obuf + lq * TW_OST + lr;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      // A[row lr][feature fb + 16c + 4lq + r], shared by both samples
      f4 at = f4zero();
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) at = mfma16(osb[4 * ks * TW_OST + 16 * c], xf[ks], at);
      float p0[4], p1[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (REV) {
          const float u = __builtin_amdgcn_fractf(at[r]);
          p0[r] = __builtin_amdgcn_cosf(u);
          p1[r] = __builtin_amdgcn_sinf(u);
        } else if (RBF) {
          float sv, cv;
          rf_sincos(at[r], &sv, &cv);
          p0[r] = cv;
          p1[r] = sv;
        } else {
          p0[r] = fmaxf(at[r], 0.f);
          p1[r] = 0.f;
        }
      }
      // F^T[i = 8 s + o][row lr] += W_s[feature][o] Phi[row lr][feature], K = the 4 features of
      // k-step r (lane group lq holds feature fb + 16c + 4lq + r)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        acc = mfma16(wl[(16 * c + r) * PST], p0[r], acc);
        if (RBF) acs = mfma16(wl[(64 + 16 * c + r) * PST], p1[r], acs);
      }
    }
    if (blk + 1 < nb) stage_store(buf ^ 1, fb + 64);
    __syncthreads();
  }
  // acc[rr] = F_s[row lr][o] / c for i = 4 lq + rr: s = lq >> 1, o = 4 (lq & 1) + rr
  float* fs = (lq >> 1) ? ftw1 : ftw0;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int o = 4 * (lq & 1) + rr;
    if (o < g) fs[lr * T.ftst + o] = cl * (acc[rr] + acs[rr]);
  }
  __syncthreads();  // both samples' F tiles complete before layer 1 reads its x fragments
}

// Per-wave timeline of the tile kernel for a separate diagnostic build (-DDGPRF_PSTAMPS, never in
// the product): slot 0 = s_memrealtime at entry, 7 = s_memtime at entry, 1..4 = s_memtime after
// each layer, 6 = s_memrealtime at exit, 5 = HW_ID | XCC_ID << 32.
#ifdef DGPRF_PSTAMPS
// DGPRF_PST_REAL: the per-layer stamps (slots 1..4, 7) in s_memrealtime ticks (100 MHz) instead of
// shader cycles, to tell clock changes from work changes
#ifdef DGPRF_PST_REAL
#define PST_CLK() __builtin_amdgcn_s_memrealtime()
#else
#define PST_CLK() __builtin_amdgcn_s_memtime()
#endif
__device__ unsigned long long g_pred_stamps[1 << 20];
#define DGPRF_PST(i, v)                                                        \
  do {                                                                         \
    const int64_t wid_ = (int64_t)blockIdx.x * TWW + (threadIdx.x >> 6);       \
    if ((threadIdx.x & 63) == 0 && wid_ * 8 + 7 < (1 << 20))                   \
      g_pred_stamps[wid_ * 8 + (i)] = (v);                                     \
  } while (0)
#else
#define DGPRF_PST(i, v) \
  do {                  \
  } while (0)
#endif

// WIDE: layer 0 reads a precomputed A_1 (separate instantiations keep the common kernels' registers);
// g > 16 instances (NOTMAX > 1) are budgeted for 2 waves/SIMD: at 4 they spilled ~300 VGPRs.
// NOTMAX = 0: the lean instance for models whose layers all have g <= 8 and d <= 8 (config 2): only
// the G8 / g == 1 bodies with two k-steps, a G8-sized W ring, and a register budget for
// TILE_LEAN_WAVES waves per SIMD (so a 1e5-row set fits about one round of workgroups).
template <int NOTMAX, int JW, int JO, int TPW, bool WIDE>
__global__ __launch_bounds__(TW_THREADS)
__attribute__((amdgpu_waves_per_eu(NOTMAX == 0 ? TILE_LEAN_WAVES
                                               : ((TPW == 1 && NOTMAX == 1) ? TILE_WAVES : 2))))
void k_forward_tiles(
    const dgprf_plan_t pl, const float* __restrict__ theta, const float* __restrict__ omega,
    const float* __restrict__ der, const float* __restrict__ X, const float* __restrict__ Y,
    const int y_cols, const int64_t n, const FOut fo, float* __restrict__ logp_out,
    float* __restrict__ se_out, float* __restrict__ lse_m, float* __restrict__ lse_s,
    float* __restrict__ se_sum, const float* __restrict__ a0, const int64_t row_begin_,
    const int64_t row_end_) {
  // rows [row_begin, row_end) of the n-row set; a0 = A_1 of those rows for a wide first layer
  // (the other instantiations always cover all n rows in one launch: constants, no extra registers)
  const int64_t row_begin = WIDE ? row_begin_ : 0, row_end = WIDE ? row_end_ : n;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const TileLds T = tile_lds(pl, NOTMAX, JO, TPW, WIDE);
  const int chain = blockIdx.y;
  const int64_t ochain = pl.hyp_per_chain ? (int64_t)chain * pl.omega_total : 0;
  const int64_t dchain = pl.hyp_per_chain ? (int64_t)chain * pl.der_total : 0;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, lr = lane & 15, lq = lane >> 4;
  const int64_t wrow0 = row_begin + (int64_t)blockIdx.x * TW_ROWS * TPW + wave * TR * TPW;
  float* xin = smem + T.xin_off + wave * TPW * TR * T.xin_st;
  float* ftw = smem + T.f_off + wave * round4(TPW * TR * T.ftst);
  const float* Wc = theta + ((int64_t)blockIdx.z * pl.n_chains + chain) * pl.w_total;
  const int L = pl.n_layers;
  DGPRF_PST(0, __builtin_amdgcn_s_memrealtime());
  DGPRF_PST(7, PST_CLK());
  DGPRF_PST(5, (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4) |
                   ((unsigned long long)__builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20) << 32));
  // this wave's X rows (zero past n)
  for (int e = lane; e < TPW * TR * T.xin_st; e += 64) {
    const int r = e / T.xin_st, k = e - r * T.xin_st;
    const int64_t b = wrow0 + r;
    xin[e] = (!WIDE && b < row_end && k < pl.d_in) ? X[b * pl.d_in + k] : 0.f;
  }
  for (int e = lane; e < TPW * TR * T.ftst; e += 64) ftw[e] = 0.f;
  __syncthreads();
  if (L < 4) DGPRF_PST(4, PST_CLK());  // input rows staged
  for (int layer = 0; layer < L; ++layer) {
    const float* __restrict__ om = omega + ochain + pl.omega_off[layer];
    const float* __restrict__ W = Wc + pl.w_off[layer];
    const float cl = der[dchain + layer];
    const int g = pl.n_gp[layer], NOT = (g + 15) >> 4;
    const float* arow0 = (WIDE && layer == 0) ? a0 + (wrow0 - row_begin) * (int64_t)pl.n_rf[0] : nullptr;
    const bool rbf = pl.kind[layer] == DGPRF_RBF, ks2 = pl.d[layer] <= 8 || arow0;
    float* fout = fo.p[layer] ? fo.p[layer] + (int64_t)chain * n * g : nullptr;
#define DGPRF_TL(NT, RB, G1_, G8_)                                                                     \
  do {                                                                                              \
    if (ks2)                                                                                        \
      tile_layer<NT, RB, G1_, G8_, JW, JO, 2, TPW>(pl, layer, W, om, cl, T, smem, xin, ftw, lr, lq, wrow0, \
                                              row_end, fout, arow0);                                \
    else                                                                                            \
      tile_layer<NT, RB, G1_, G8_, JW, JO, 4 * JO, TPW>(pl, layer, W, om, cl, T, smem, xin, ftw, lr, lq,  \
                                                   wrow0, row_end, fout);                           \
  } while (0)
    if (NOTMAX == 0) {  // lean: g <= 8 and d <= 8 on every layer (host-checked)
      if (g == 1) {
        if (rbf) tile_layer<1, true, true, false, JW, JO, 2, TPW, false, true>(pl, layer, W, om, cl, T, smem, xin, ftw, lr, lq, wrow0, row_end, fout);
        else tile_layer<1, false, true, false, JW, JO, 2, TPW, false, true>(pl, layer, W, om, cl, T, smem, xin, ftw, lr, lq, wrow0, row_end, fout);
      } else {
        if (rbf) tile_layer<1, true, false, true, JW, JO, 2, TPW, false, true>(pl, layer, W, om, cl, T, smem, xin, ftw, lr, lq, wrow0, row_end, fout);
        else tile_layer<1, false, false, true, JW, JO, 2, TPW, false, true>(pl, layer, W, om, cl, T, smem, xin, ftw, lr, lq, wrow0, row_end, fout);
      }
    } else if (g == 1) {
      if (rbf) DGPRF_TL(1, true, true, false);
      else DGPRF_TL(1, false, true, false);
    } else if (g <= 8) {
      if (rbf) DGPRF_TL(1, true, false, true);
      else DGPRF_TL(1, false, false, true);
    } else if (NOT == 1) {
      if (rbf) DGPRF_TL(1, true, false, false);
      else DGPRF_TL(1, false, false, false);
    } else if (NOTMAX >= 2 && NOT == 2) {
      if (rbf) DGPRF_TL((NOTMAX >= 2 ? 2 : 1), true, false, false);
      else DGPRF_TL((NOTMAX >= 2 ? 2 : 1), false, false, false);
    } else if (NOTMAX >= 4) {
      if (rbf) DGPRF_TL((NOTMAX >= 4 ? 4 : 1), true, false, false);
      else DGPRF_TL((NOTMAX >= 4 ? 4 : 1), false, false, false);
    }
#undef DGPRF_TL
    if (layer < 4) DGPRF_PST(1 + layer, PST_CLK());
  }
  // likelihood per row: lanes 0..15 of each wave, row lr of each of the wave's tiles
  const bool want_lik = logp_out || se_out || lse_m;
  for (int t = 0; t < TPW; ++t) {
    const int64_t b = wrow0 + t * TR + lr;
    if (want_lik && lq == 0 && b < row_end) {
      const int g = pl.n_gp[L - 1];
      const float* f = ftw + (t * TR + lr) * T.ftst;
      const float* y = Y + b * y_cols;
      float lp = 0.f, se = 0.f;
      if (pl.likelihood == DGPRF_LIK_GAUSSIAN) {
        const float var = der[dchain + DGPRF_MAX_LAYERS];
        const float logvar = logf(var);
        for (int o = 0; o < g; ++o) {
          const float diff = y[o] - f[o];
          lp += -0.5f * (LOG_2PI + logvar + diff * diff / var);
          se += diff * diff;
        }
        se = se / (float)g;  // reduce_mean over outputs (regression_model.py:46)
      } else {
        float mx = -INFINITY;
        for (int o = 0; o < g; ++o) mx = fmaxf(mx, f[o]);
        float s = 0.f;
        for (int o = 0; o < g; ++o) s += expf(f[o] - mx);
        // int32(Y[:, 0]) (likelihoods/softmax.py:14); a label outside [0, g) scores NaN (TF raises)
        const int lab = (int)y[0];
        const bool lab_ok = lab >= 0 && lab < g;
        lp = lab_ok ? f[lab] - (mx + logf(s)) : __builtin_nanf("");
      }
      const int64_t idx = (int64_t)chain * n + b;
      // blockIdx.z = sample of a multi-sample launch: its outputs [sample][chain][n]
      const int64_t oidx = (int64_t)blockIdx.z * pl.n_chains * n + idx;
      if (logp_out) logp_out[oidx] = lp;
      if (se_out) se_out[oidx] = se;
      if (lse_m) lse_fold1(lse_m, lse_s, se_sum, idx, lp, se);
    }
  }
  DGPRF_PST(6, __builtin_amdgcn_s_memrealtime());
}

// Posterior-predictive scoring of one pair of samples of every chain (thetas [2][C][w_total]; two =
// false: one sample) for lean models (every layer d, g <= 8; config 2): layer 0 once for the pair
// (tile_layer0_pair), layers >= 1 and the likelihood per sample, each sample folded into the
// chain's online log-sum-exp accumulators in sample order (experiments/utils_training.py:79-85).
// A workgroup covers 64 test rows of one chain, so each accumulator element has one writer.
// Same register budget as the lean one-sample instance.
__global__ __launch_bounds__(TW_THREADS) __attribute__((amdgpu_waves_per_eu(TILE_LEAN_WAVES)))
void k_forward_pairs(const dgprf_plan_t pl, const float* __restrict__ thetas, const int n_samples,
                     const float* __restrict__ omega, const float* __restrict__ der,
                     const float* __restrict__ X, const float* __restrict__ Y, const int y_cols,
                     const int64_t n, float* __restrict__ lse_m, float* __restrict__ lse_s,
                     float* __restrict__ se_sum, float* __restrict__ lp_out,
                     float* __restrict__ se_out) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const TileLds T = tile_lds(pl, 0, 1, 1, false, 2);
  const int chain = blockIdx.y, C = pl.n_chains;
  // pair blockIdx.z: samples s0 = 2 z and s0 + 1 (when s0 + 1 < n_samples) of thetas
  const int s0 = 2 * (int)blockIdx.z, two = s0 + 1 < n_samples ? 1 : 0;
  const int64_t ochain = pl.hyp_per_chain ? (int64_t)chain * pl.omega_total : 0;
  const int64_t dchain = pl.hyp_per_chain ? (int64_t)chain * pl.der_total : 0;
  // the wave index through readfirstlane: the wave's LDS tiles / row base are SGPR values, not
  // per-lane registers live through both samples' layers
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, lr = lane & 15, lq = lane >> 4;
  const int64_t wrow0 = (int64_t)blockIdx.x * TW_ROWS + wave * TR;
  float* xin = smem + T.xin_off + wave * TR * T.xin_st;
  float* ftw0 = smem + T.f_off + (2 * wave) * round4(TR * T.ftst);
  float* ftw1 = smem + T.f_off + (2 * wave + 1) * round4(TR * T.ftst);
  const int L = pl.n_layers;
  DGPRF_PST(0, __builtin_amdgcn_s_memrealtime());
  DGPRF_PST(7, PST_CLK());
  for (int e = lane; e < TR * T.xin_st; e += 64) {
    const int r = e / T.xin_st, k = e - r * T.xin_st;
    const int64_t b = wrow0 + r;
    xin[e] = (b < n && k < pl.d_in) ? X[b * pl.d_in + k] : 0.f;
  }
  for (int e = lane; e < TR * T.ftst; e += 64) ftw0[e] = ftw1[e] = 0.f;
  __syncthreads();
  const float* om0 = omega + ochain + pl.omega_off[0];
  {
    const float* W0 = thetas + ((int64_t)s0 * C + chain) * pl.w_total;
    const float* W1 = two ? W0 + (int64_t)C * pl.w_total : W0;
    if (pl.kind[0] == DGPRF_RBF)
      tile_layer0_pair<true>(pl, W0, W1, om0, der[dchain], T, smem, xin, ftw0, ftw1, lr, lq);
    else
      tile_layer0_pair<false>(pl, W0, W1, om0, der[dchain], T, smem, xin, ftw0, ftw1, lr, lq);
    DGPRF_PST(1, PST_CLK());
    // unrolled: each sample's copy of layers >= 1 keeps only its own state live (a loop over the
    // two samples spilled 5 VGPRs at the 96-register budget; unrolled: 92, none spilled)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (j == 1 && !two) break;
      float* ftw = j ? ftw1 : ftw0;
      const float* Wc = j ? W1 : W0;
      for (int layer = 1; layer < L; ++layer) {
        const float* __restrict__ om = omega + ochain + pl.omega_off[layer];
        const float* __restrict__ W = Wc + pl.w_off[layer];
        const float cl = der[dchain + layer];
        const bool rbf = pl.kind[layer] == DGPRF_RBF;
        if (pl.n_gp[layer] == 1) {
          if (rbf) tile_layer<1, true, true, false, 1, 1, 2, 1, false, true>(pl, layer, W, om, cl, T, smem, xin, ftw, lr, lq, wrow0, n, nullptr);
          else tile_layer<1, false, true, false, 1, 1, 2, 1, false, true>(pl, layer, W, om, cl, T, smem, xin, ftw, lr, lq, wrow0, n, nullptr);
        } else {
          if (rbf) tile_layer<1, true, false, true, 1, 1, 2, 1, false, true>(pl, layer, W, om, cl, T, smem, xin, ftw, lr, lq, wrow0, n, nullptr);
          else tile_layer<1, false, false, true, 1, 1, 2, 1, false, true>(pl, layer, W, om, cl, T, smem, xin, ftw, lr, lq, wrow0, n, nullptr);
        }
      }
      // likelihood of this sample, folded into the chain's accumulators (as k_forward_tiles)
      const int64_t b = wrow0 + lr;
      if (lq == 0 && b < n) {
        const int g = pl.n_gp[L - 1];
        const float* f = ftw + lr * T.ftst;
        const float* y = Y + b * y_cols;
        float lp = 0.f, se = 0.f;
        if (pl.likelihood == DGPRF_LIK_GAUSSIAN) {
          const float var = der[dchain + DGPRF_MAX_LAYERS];
          const float logvar = logf(var);
          for (int o = 0; o < g; ++o) {
            const float diff = y[o] - f[o];
            lp += -0.5f * (LOG_2PI + logvar + diff * diff / var);
            se += diff * diff;
          }
          se = se / (float)g;
        } else {
          float mx = -INFINITY;
          for (int o = 0; o < g; ++o) mx = fmaxf(mx, f[o]);
          float sm = 0.f;
          for (int o = 0; o < g; ++o) sm += expf(f[o] - mx);
          const int lab = (int)y[0];
          lp = (lab >= 0 && lab < g) ? f[lab] - (mx + logf(sm)) : __builtin_nanf("");
        }
        const int64_t idx = (int64_t)chain * n + b;
        if (lp_out) {  // every pair of the call in one launch: [sample][chain][n], folded after
          const int64_t o = (int64_t)(s0 + j) * C * n + idx;
          lp_out[o] = lp;
          if (se_out) se_out[o] = se;
        } else {
          lse_fold1(lse_m, lse_s, se_sum, idx, lp, se);
        }
      }
      DGPRF_PST(2 + j, PST_CLK());
    }
  }
  DGPRF_PST(6, __builtin_amdgcn_s_memrealtime());
}

// The per-row log p / squared errors of n_samples samples ([sample][chain][n], one multi-pair
// launch) folded into the accumulators in sample order — the same sequence of lse_fold1 steps the
// one-pair-per-launch path takes, so the same bits.
__global__ __launch_bounds__(256) void k_lse_fold_samples(const float* __restrict__ lp,
                                                          const float* __restrict__ se,
                                                          int n_samples, int64_t cn,
                                                          float* __restrict__ lse_m,
                                                          float* __restrict__ lse_s,
                                                          float* __restrict__ se_sum) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= cn) return;
  for (int j = 0; j < n_samples; ++j)
    lse_fold1(lse_m, lse_s, se_sum, idx, lp[j * cn + idx], se ? se[j * cn + idx] : 0.f);
}

}  // namespace

#ifdef DGPRF_PSTAMPS
extern "C" int dgprf_debug_read_pred_stamps(unsigned long long* host, long long n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_pred_stamps), (size_t)n * 8, 0,
                             hipMemcpyDeviceToHost);
}
#endif

namespace dgprf {

// compute units of the current device (queried once; 256 on MI355X)
static int device_cus() {
  static const int cus = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return cus;
}

ForwardCfg forward_cfg(const dgprf_plan_t& pl, int64_t n, int n_samples) {
  ForwardCfg c;
  // wide first layer (d_1 > 32, e.g. 784 pixels): A_1 = X Omega_1 by the tiled GEMM
  // (k_step_agemm), in row chunks of caller-owned scratch, read by layer 0 instead of a d-long
  // k-step loop per feature chunk (needs one Omega_1 for all chains)
  c.wide0 = pl.fwd_path != DGPRF_FWD_NO_AGEMM && pl.d[0] > 32 &&
            (!pl.hyp_per_chain || pl.n_chains == 1) && pl.n_rf[0] % 4 == 0 &&
            (int64_t)pl.d[0] * pl.n_rf[0] < ((int64_t)1 << 29);
  // tile kernel: d <= 32 (layer 0 exempt when wide0 and no input concatenation), g <= 64,
  // R % 4 == 0 in every layer
  bool tile_ok = (pl.d_in <= 32) || (c.wide0 && !pl.input_cat);
  bool small = true;  // d <= 32 and g <= 16 in every layer: the 16-wave row kernel applies
  for (int l = 0; l < pl.n_layers; ++l) {
    tile_ok = tile_ok && (pl.d[l] <= 32 || (l == 0 && c.wide0)) && pl.n_gp[l] <= 64 &&
              pl.n_rf[l] % 4 == 0 && (int64_t)2 * pl.n_rf[l] * pl.n_gp[l] < ((int64_t)1 << 29);
    small = small && pl.d[l] <= 32 && pl.n_gp[l] <= 16;
  }
  // the tile kernel gives each 16-row tile ONE wave through all layers: below FWD_TILE_MIN_ROWS
  // rows it leaves most SIMDs idle, and the row kernel with 16 waves per tile (each a sixteenth
  // of every layer's features, F partials summed in LDS) covers the chip instead
  constexpr int64_t FWD_TILE_MIN_ROWS = 16384, FWD_TILE_MANY_ROWS = 65536;
  const bool few = n < FWD_TILE_MIN_ROWS;
  // layers with g > 16 run the tile kernel at 2 waves per SIMD (its 2-4 output tiles per wave do
  // not fit 4): the 4-wave row kernel is faster at every measured size (config 4: 10k / 20k / 40k
  // test rows 1,072 / 1,923 / 3,716 us vs 1,167 / 2,321 / 4,026 us on the tile kernel)
  bool wide_g = false;
  for (int l = 0; l < pl.n_layers; ++l) wide_g = wide_g || pl.n_gp[l] > 16;
  switch (pl.fwd_path) {
    case DGPRF_FWD_ROWS: c.tiles = false; c.rows_waves = 4; break;
    case DGPRF_FWD_ROWS16: c.tiles = false; c.rows_waves = small ? 16 : 4; break;
    case DGPRF_FWD_ROWS8: c.tiles = false; c.rows_waves = small ? 8 : 4; break;
    case DGPRF_FWD_TILE: c.tiles = tile_ok; c.rows_waves = 4; break;
    // small sets: 16 waves per tile while every tile has a CU of its own; past that (config 3:
    // 286 tiles) two 8-wave workgroups share a CU (4,573 rows: 43.1 vs 47.8 us with 16 waves)
    default:
      // a launch of many rows in all — n rows x the samples (grid.z) x the chains (grid.y) of one
      // launch — fills the chip with one-wave tiles however few rows one sample has, and the tile
      // kernel's per-tile work is the cheaper one there (config 3, 4,573 rows, 60 samples: 15.9 vs
      // 21.7 us per sample; config 4, 10,000 rows with g = 30: 289 vs 385 us; the row kernels win
      // below about 40k-70k rows in all: config 3 x 8 samples 22.4 vs 24.0 us, config 4 x 2 samples
      // 424 vs 494 us)
      if ((int64_t)n * n_samples * pl.n_chains >= FWD_TILE_MANY_ROWS) {
        c.tiles = tile_ok;
        c.rows_waves = 4;
        break;
      }
      c.tiles = tile_ok && !few && !wide_g;
      c.rows_waves = few && small ? ((n + TR - 1) / TR > device_cus() ? 8 : 16) : 4;
      break;
  }
  // past one tile per CU a CU runs two tiles anyway: for ONE sample of one chain, one 16-wave
  // workgroup over two tiles fetches each W / Omega fragment once for both (instead of two 8-wave
  // workgroups fetching the model twice): config 3's 4,573 rows 36.4 vs 40.0 us.  A launch of
  // several samples or chains keeps the 8-wave workgroups (2 / 4 samples: 30.3 vs 35.8 / 23.7 vs
  // 26.6 us per sample).  DGPRF_FWD_ROWS8 keeps the two-workgroup form.
  c.rows_tt = 1;
  if (pl.fwd_path == DGPRF_FWD_AUTO && c.rows_waves == 8 && !c.wide0 && n_samples * pl.n_chains == 1) {
    c.rows_waves = 16;
    c.rows_tt = 2;
  }
  // chunks are whole 64-row tile-kernel workgroups: every wave of the last workgroup reads its 16
  // A_1 rows (rows past n included, their outputs discarded), so the scratch covers align64 rows
  const int64_t R0 = pl.n_rf[0];
  int64_t cap = (((int64_t)1 << 26) / R0) / TW_ROWS * TW_ROWS;
  if (pl.agemm_chunk_rows > 0)
    cap = std::max<int64_t>(TW_ROWS, pl.agemm_chunk_rows / TW_ROWS * TW_ROWS);
  c.chunk = c.wide0 ? std::max<int64_t>(TW_ROWS, std::min<int64_t>(cap, (n + TW_ROWS - 1) / TW_ROWS * TW_ROWS))
                    : n;
  c.scratch_floats = c.wide0 && n > 0 ? c.chunk * R0 : 0;
  return c;
}

hipError_t launch_forward_rows(const dgprf_plan_t& pl, const float* theta, const float* omega,
                               const float* der, const float* X, const float* Y, int y_cols,
                               int64_t n, float* const* f_out, float* logp, float* se,
                               float* lse_m, float* lse_s, float* se_sum, float* scratch,
                               hipStream_t s, const float* a1_full, int n_samples,
                               int path_samples) {
  if (n <= 0) return hipSuccess;
  // n_samples > 1: theta holds that many samples ([n_samples][C][w_total]), one per grid.z, and
  // logp / se receive [n_samples][C][n] (no in-kernel fold: the caller folds in sample order)
  if (n_samples > 1 && (lse_m || (f_out && f_out[0]))) return hipErrorInvalidValue;
  FOut fo;
  for (int l = 0; l < DGPRF_MAX_LAYERS; ++l) fo.p[l] = (f_out && l < pl.n_layers) ? f_out[l] : nullptr;
  bool smalld = true;
  int notmax = 1;
  for (int l = 0; l < pl.n_layers; ++l) {
    smalld = smalld && pl.d[l] <= 32;
    notmax = max(notmax, (pl.n_gp[l] + 15) >> 4);
  }
  const ForwardCfg cfg = forward_cfg(pl, n, path_samples > 0 ? path_samples : n_samples);
  const bool wide0 = cfg.wide0, tiles = cfg.tiles;
  // a caller-resident A_1 of every row: one chunk, no GEMM
  const bool res = wide0 && a1_full;
  const int64_t chunk = res ? n : cfg.chunk, R0 = pl.n_rf[0];
  float* a0 = res ? const_cast<float*>(a1_full) : (wide0 ? scratch : nullptr);
  if (wide0 && !a0) return hipErrorInvalidValue;
  hipError_t err = hipSuccess;
  for (int64_t r0 = 0; r0 < n && err == hipSuccess; r0 += chunk) {
    const int64_t r1 = std::min(n, r0 + chunk);
    if (wide0 && !res) {
      err = launch_agemm(X + r0 * pl.d_in, r1 - r0, pl.d_in, pl.d[0], omega + pl.omega_off[0],
                         (int)R0, a0, s);
      if (err != hipSuccess) break;
    }
    const int64_t nr = r1 - r0;
    if (tiles) {
      int gmax = 1, dmax = 1;
      for (int l = 0; l < pl.n_layers; ++l) {
        gmax = max(gmax, pl.n_gp[l]);
        if (!(l == 0 && wide0)) dmax = max(dmax, pl.d[l]);  // Omega rows staged per block
      }
      const int njw = gmax <= 8 ? 1 : (gmax <= 16 ? 2 : (gmax <= 32 ? 4 : 8));  // >= 32 g / 256
      // >= 16 d / 256; the wide-g instances are compiled with JO = 2 only (host and kernel must
      // size the LDS ring identically)
      const int njo = (dmax <= 16 && njw <= 2) ? 1 : 2;
      int ntm = njw <= 2 ? 1 : (njw == 4 ? 2 : 4);
      constexpr int tpw = TILE_TPW_DEFAULT;
      bool lean = !wide0 && tpw == 1 && njw == 1 && njo == 1;
      for (int l = 0; l < pl.n_layers; ++l) lean = lean && pl.n_gp[l] <= 8 && pl.d[l] <= 8;
      if (lean) ntm = 0;
      const TileLds T = tile_lds(pl, ntm, njo, tpw, wide0);
      dim3 tgrid((unsigned)((nr + TW_ROWS * tpw - 1) / (TW_ROWS * tpw)), pl.n_chains, n_samples);
      const size_t tl = (size_t)T.total * sizeof(float);
#define DGPRF_TILE_LAUNCH1(NM, J, JO, TP, WD)                                                      \
  do {                                                                                             \
    set_lds_limit((const void*)k_forward_tiles<NM, J, JO, TP, WD>, tl);                            \
    hipLaunchKernelGGL((k_forward_tiles<NM, J, JO, TP, WD>), tgrid, dim3(TW_THREADS), tl, s, pl,   \
                       theta, omega, der, X, Y, y_cols, n, fo, logp, se, lse_m, lse_s, se_sum, a0, \
                       r0, r1);                                                                    \
  } while (0)
#define DGPRF_TILE_LAUNCH(NM, J, JO)                                                               \
  do {                                                                                             \
    if (wide0) DGPRF_TILE_LAUNCH1(NM, J, JO, 1, true);                                             \
    else DGPRF_TILE_LAUNCH1(NM, J, JO, tpw, false);                                                \
  } while (0)
      if (lean) {
        DGPRF_TILE_LAUNCH1(0, 1, 1, 1, false);
      } else if (njw == 1) {
        if (njo == 1) DGPRF_TILE_LAUNCH(1, 1, 1);
        else DGPRF_TILE_LAUNCH(1, 1, 2);
      } else if (njw == 2) {
        if (njo == 1) DGPRF_TILE_LAUNCH(1, 2, 1);
        else DGPRF_TILE_LAUNCH(1, 2, 2);
      } else if (njw == 4) {
        DGPRF_TILE_LAUNCH(2, 4, 2);
      } else {
        DGPRF_TILE_LAUNCH(4, 8, 2);
      }
#undef DGPRF_TILE_LAUNCH
#undef DGPRF_TILE_LAUNCH1
    } else {
      const int nwr = cfg.rows_waves, tt = cfg.rows_tt;
      const size_t lds = (size_t)fwd_lds(pl, nwr, tt).total * sizeof(float);
      dim3 grid((unsigned)((nr + TR * tt - 1) / (TR * tt)), pl.n_chains, n_samples);
#define DGPRF_FWD_LAUNCH_W(S, NM, NWR_)                                                             \
  do {                                                                                             \
    set_lds_limit((const void*)k_forward_rows<S, NM, NWR_>, lds);                                  \
    hipLaunchKernelGGL((k_forward_rows<S, NM, NWR_>), grid, dim3(64 * NWR_), lds, s, pl, theta,    \
                       omega, der, X, Y, y_cols, n, fo, logp, se, lse_m, lse_s, se_sum, a0, r0, r1); \
  } while (0)
#define DGPRF_FWD_LAUNCH(S, NM) DGPRF_FWD_LAUNCH_W(S, NM, 4)
      if (smalld && tt == 2) {  // g <= 16, no wide first layer (forward_cfg)
        set_lds_limit((const void*)k_forward_rows<true, 1, 16, 2>, lds);
        hipLaunchKernelGGL((k_forward_rows<true, 1, 16, 2>), grid, dim3(64 * 16), lds, s, pl, theta,
                           omega, der, X, Y, y_cols, n, fo, logp, se, lse_m, lse_s, se_sum, a0, r0, r1);
      } else if (smalld && nwr == 16 && (nr + TR - 1) / TR <= device_cus()) {  // one workgroup per CU: 4 waves per SIMD
        set_lds_limit((const void*)k_forward_rows<true, 1, 16, 1, 4>, lds);
        hipLaunchKernelGGL((k_forward_rows<true, 1, 16, 1, 4>), grid, dim3(64 * 16), lds, s, pl, theta,
                           omega, der, X, Y, y_cols, n, fo, logp, se, lse_m, lse_s, se_sum, a0, r0, r1);
      } else if (smalld && nwr == 16) {  // g <= 16 (forward_cfg)
        DGPRF_FWD_LAUNCH_W(true, 1, 16);
      } else if (smalld && nwr == 8) {
        DGPRF_FWD_LAUNCH_W(true, 1, 8);
      } else if (smalld) {
        if (notmax == 1) DGPRF_FWD_LAUNCH(true, 1);
        else if (notmax == 2) DGPRF_FWD_LAUNCH(true, 2);
        else DGPRF_FWD_LAUNCH(true, 4);
      } else {
        if (notmax == 1) DGPRF_FWD_LAUNCH(false, 1);
        else if (notmax == 2) DGPRF_FWD_LAUNCH(false, 2);
        else DGPRF_FWD_LAUNCH(false, 4);
      }
#undef DGPRF_FWD_LAUNCH
#undef DGPRF_FWD_LAUNCH_W
    }
    err = hipGetLastError();
  }
  return err;
}

// The pair kernel applies where the one-sample path would run the lean tile instance.
bool forward_pairs_ok(const dgprf_plan_t& pl, int64_t n, int n_samples) {
  const ForwardCfg cfg = forward_cfg(pl, n, n_samples);
  if (!cfg.tiles || cfg.wide0 || TILE_TPW_DEFAULT != 1) return false;
  for (int l = 0; l < pl.n_layers; ++l)
    if (pl.n_gp[l] > 8 || pl.d[l] > 8) return false;
  return true;
}

hipError_t launch_forward_samples(const dgprf_plan_t& pl, const float* thetas, int n_samples,
                                  const float* omega, const float* der, const float* X,
                                  const float* A1, const float* Y, int y_cols, int64_t n, float* lse_m,
                                  float* lse_s, float* se_sum, float* scratch,
                                  int64_t scratch_floats, hipStream_t s) {
  if (n <= 0 || n_samples <= 0) return hipSuccess;
  // 32-bit buffer offsets across two samples' W
  const bool off_ok = ((int64_t)pl.n_chains * pl.w_total + 2 * (int64_t)pl.n_rf[0] * pl.n_gp[0]) * 4 <
                      ((int64_t)1 << 31);
  if (!off_ok || !forward_pairs_ok(pl, n, n_samples)) {
    const int64_t cn = (int64_t)pl.n_chains * n;
    const int64_t need = forward_samples_scratch(pl, n, n_samples);
    if (need > 0 && scratch && scratch_floats >= need && (A1 || !forward_cfg(pl, n).wide0)) {
      // every sample in one launch (grid.z = sample): a small test set's launch leaves most of the
      // chip idle (config 3: 143 workgroups; config 4: 2.4 rounds of 625), several fill it; the
      // per-row log p / se go to scratch and the fold applies them in sample order
      float* lp = scratch;
      float* se = se_sum ? scratch + (int64_t)n_samples * cn : nullptr;
      hipError_t e = launch_forward_rows(pl, thetas, omega, der, X, Y, y_cols, n, nullptr, lp, se,
                                         nullptr, nullptr, nullptr, nullptr, s, A1, n_samples);
      if (e != hipSuccess) return e;
      hipLaunchKernelGGL(k_lse_fold_samples, dim3((unsigned)((cn + 255) / 256)), dim3(256), 0, s,
                         lp, se, n_samples, cn, lse_m, lse_s, se_sum);
      return hipGetLastError();
    }
    for (int j = 0; j < n_samples; ++j) {  // one launch per sample (sample order)
      const hipError_t e = launch_forward_rows(pl, thetas + (int64_t)j * pl.n_chains * pl.w_total,
                                               omega, der, X, Y, y_cols, n, nullptr, nullptr,
                                               nullptr, lse_m, lse_s, se_sum, scratch, s, A1, 1,
                                               n_samples);  // the one-launch form's kernel
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  const TileLds T = tile_lds(pl, 0, 1, 1, false, 2);
  const size_t tl = (size_t)T.total * sizeof(float);
  const unsigned tiles = (unsigned)((n + TW_ROWS - 1) / TW_ROWS);
  set_lds_limit((const void*)k_forward_pairs, tl);
  const int64_t cn = (int64_t)pl.n_chains * n;
  const int pairs = (n_samples + 1) / 2;
  if (pairs > 1 && scratch && scratch_floats >= forward_samples_scratch(pl, n, n_samples)) {
    // every pair in ONE launch (grid.z = pair): a launch of one pair leaves the chip part-empty for
    // its last ~40 % (1.22 rounds of resident waves at 1e5 rows); its rows' log p go to scratch
    // and one fold kernel applies them in sample order
    float* lp = scratch;
    float* se = se_sum ? scratch + (int64_t)n_samples * cn : nullptr;
    hipLaunchKernelGGL(k_forward_pairs, dim3(tiles, pl.n_chains, pairs), dim3(TW_THREADS), tl, s,
                       pl, thetas, n_samples, omega, der, X, Y, y_cols, n, lse_m, lse_s, se_sum, lp,
                       se);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_lse_fold_samples, dim3((unsigned)((cn + 255) / 256)), dim3(256), 0, s, lp,
                       se, n_samples, cn, lse_m, lse_s, se_sum);
    return hipGetLastError();
  }
  for (int p = 0; p < pairs; ++p) {  // one launch per pair of samples, folded in place
    hipLaunchKernelGGL(k_forward_pairs, dim3(tiles, pl.n_chains, 1), dim3(TW_THREADS), tl, s, pl,
                       thetas + (int64_t)2 * p * pl.n_chains * pl.w_total,
                       2 * p + 1 < n_samples ? 2 : 1, omega, der, X, Y, y_cols, n, lse_m, lse_s,
                       se_sum, nullptr, nullptr);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// scratch floats the one-launch form of launch_forward_samples needs: log p (and, Gaussian, the
// squared error) of every sample's rows; 0 when that form does not apply
int64_t forward_samples_scratch(const dgprf_plan_t& pl, int64_t n, int n_samples) {
  if (n <= 0) return 0;
  const int64_t per = (int64_t)pl.n_chains * n * (pl.likelihood == DGPRF_LIK_GAUSSIAN ? 2 : 1);
  if (forward_pairs_ok(pl, n, n_samples)) return n_samples >= 3 ? n_samples * per : 0;
  // one-sample kernels: all samples in one launch (launch_forward_samples takes that form unless
  // a wide first layer's A_1 would come in scratch chunks, i.e. without a resident projection)
  return n_samples >= 2 ? n_samples * per : 0;
}

size_t forward_rows_lds_bytes(const dgprf_plan_t& pl) {
  return (size_t)fwd_lds(pl).total * sizeof(float);
}

hipError_t launch_lse_finalize(const float* lse_m, const float* lse_s, const float* se_sum,
                               int parts, int64_t n, double s_total, float log_y_std, float y_std,
                               float* lse_out, double* out, hipStream_t s) {
  hipLaunchKernelGGL(k_lse_finalize, dim3(1), dim3(1024), 0, s, lse_m, lse_s, se_sum, parts, n,
                     s_total, log_y_std, y_std, lse_out, out);
  return hipGetLastError();
}

hipError_t launch_rf_features(int kind, const float* X, int64_t n, int d, const float* omega, int R,
                              const float* c, float* phi, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  dim3 grid((unsigned)((n + TR - 1) / TR), (unsigned)((R + NW * 16 - 1) / (NW * 16)));
  hipLaunchKernelGGL(k_rf_features, grid, dim3(256), 0, s, kind, X, n, d, omega, R, c, phi);
  return hipGetLastError();
}

hipError_t launch_gp_matmul(const float* phi, int64_t n, int P, const float* W, int g, float* F,
                            hipStream_t s) {
  if (n <= 0) return hipSuccess;
  // 32-bit buffer offsets within one 16-row tile of Phi and within W
  if ((int64_t)16 * P >= ((int64_t)1 << 29) || (int64_t)P * g >= ((int64_t)1 << 29))
    return hipErrorInvalidValue;
  dim3 grid((unsigned)((n + 15) / 16), (unsigned)((g + 15) / 16));
  hipLaunchKernelGGL(k_gp_matmul, grid, dim3(256), 0, s, phi, n, P, W, g, F);
  return hipGetLastError();
}

hipError_t launch_prior_w(const dgprf_plan_t& pl, const float* theta, float* out, hipStream_t s) {
  hipLaunchKernelGGL(k_prior_w, dim3(pl.n_chains), dim3(256), 0, s, pl, theta, out);
  return hipGetLastError();
}

}  // namespace dgprf
