// step_kernels.hip — one SGHMC/SGLD step of the DGP-RF sampler on gfx950.
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
//   the SGHMC update with Philox noise.  Omega/W fragments of a wave's first chunk are loaded
//   before the dependent partial sums so both latencies overlap.
#include "dgprf_internal.h"

namespace {

constexpr int NW = DGPRF_WAVES;
constexpr int TR = DGPRF_TILE_ROWS;
constexpr int NSM = DGPRF_NS_MAX;
constexpr float LOG_2PI = 1.8378770664093453f;

__device__ __forceinline__ int64_t cur_step(const StepDev& sd) {
  return *sd.step + (int64_t)sd.step_offset;
}

__host__ __device__ __forceinline__ int round4(int x) { return (x + 3) & ~3; }

// sum over the DGPRF_NS_MAX slices of a partial buffer: independent loads, fixed order.
__device__ __forceinline__ float sum_slices(const float* __restrict__ p, int64_t stride) {
  float v[NSM];
#pragma unroll
  for (int s = 0; s < NSM; ++s) v[s] = p[s * stride];
  float acc = v[0];
#pragma unroll
  for (int s = 1; s < NSM; ++s) acc += v[s];
  return acc;
}

// LDS carve of a step kernel (floats):  ridx (16 x int64) | xs [16][xst] | aux [16][auxst] | red
struct StepLds {
  int xst, aux_off, auxst, red_off, total;
};

__host__ __device__ inline StepLds step_lds(const dgprf_plan_t& pl, int layer) {
  StepLds L;
  const int d = pl.d[layer];
  L.xst = round4(d) + 1;
  L.aux_off = 32 + round4(TR * L.xst);
  L.auxst = pl.n_gp[layer] + 1;
  L.red_off = L.aux_off + round4(TR * L.auxst);
  L.total = L.red_off + NW * TR * 64;
  return L;
}

// Does layer `layer`'s X tile need dataset rows?  (layer 0, or input_cat concatenation)
__device__ __forceinline__ bool needs_rows(const dgprf_plan_t& pl, int layer) {
  return layer == 0 || pl.input_cat;
}

// Build the layer-`layer` input tile X_l[16][d_l] of batch rows row0.. into xs.
//   layer 0: minibatch rows of the dataset; layer l>0: sum over slices of F_{l-1} partials
//   (+ the dataset row for input_cat, [F | X] order of utils.py:42).
__device__ void load_x_tile(const dgprf_plan_t& pl, const StepDev& sd, int layer, int chain,
                            int row0, const int64_t* ridx, float* xs, int xst) {
  const int d = pl.d[layer], dpad = round4(d), B = pl.batch;
  const float* wsc = sd.ws + (int64_t)chain * pl.ws_chain;
  const int gp = layer > 0 ? pl.n_gp[layer - 1] : 0;
  for (int e = threadIdx.x; e < TR * dpad; e += blockDim.x) {
    const int r = e / dpad, k = e - r * dpad, b = row0 + r;
    float v = 0.f;
    if (b < B && k < d) {
      if (k < gp)
        v = sum_slices(wsc + pl.fp_off[layer - 1] + (int64_t)b * gp + k, (int64_t)B * gp);
      else
        v = sd.bd.X[ridx[r] * pl.d_in + (k - gp)];
    }
    xs[r * xst + k] = v;
  }
}

__device__ __forceinline__ void fill_ridx(const dgprf_plan_t& pl, const StepDev& sd, int chain,
                                          int row0, int64_t t, int64_t* ridx) {
  if (threadIdx.x < TR) {
    const int b = row0 + threadIdx.x;
    ridx[threadIdx.x] = (b < pl.batch) ? batch_row(sd.bd, pl.batch, chain, t, b) : 0;
  }
}

// Omega fragments of one 16-feature chunk: om_k[ks] = Omega[4ks+lq][f0+lr] (SMALLD: d <= 32).
__device__ __forceinline__ void load_om_frag(const float* __restrict__ om, int R, int d, int f0,
                                             int lr, int lq, float (&omk)[8]) {
  const int fa = f0 + lr;
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) {
    const int k = 4 * ks + lq;
    omk[ks] = (4 * ks < d && fa < R && k < d) ? om[(int64_t)k * R + fa] : 0.f;
  }
}

// A-tile from fragments.  TRANS=false: at[r] = A[row lr][f0+4lq+r]   (features in regs)
//                         TRANS=true : at[r] = A[row 4lq+r][f0+lr]   (rows in regs)
template <bool SMALLD, bool TRANS>
__device__ __forceinline__ f4 a_tile(const float* __restrict__ om, int R, int d, int f0,
                                     const float (&omk)[8], const float (&xf)[8],
                                     const float* xs, int xst, int lr, int lq) {
  f4 at = f4zero();
  if (SMALLD) {
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
      if (4 * ks < d) at = TRANS ? mfma16(xf[ks], omk[ks], at) : mfma16(omk[ks], xf[ks], at);
  } else {
    const int fa = f0 + lr;
    const bool fok = fa < R;
    const int KS = round4(d) >> 2;
    for (int ks = 0; ks < KS; ++ks) {
      const int k = 4 * ks + lq;
      const float o = (fok && k < d) ? om[(int64_t)k * R + fa] : 0.f;
      const float x = xs[lr * xst + 4 * ks + lq];
      at = TRANS ? mfma16(x, o, at) : mfma16(o, x, at);
    }
  }
  return at;
}

template <bool RBF>
__device__ __forceinline__ void features(const f4 at, float cl, float (&p0)[4], float (&p1)[4]) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (RBF) {
      float s, c;
      rf_sincos(at[r], &s, &c);
      p0[r] = cl * c;
      p1[r] = cl * s;
    } else {
      p0[r] = cl * fmaxf(at[r], 0.f);
      p1[r] = 0.f;
    }
  }
}

// W fragments for F^T += W^T Phi^T: wf[ot][r][0|1] = W[f0+4lq+r (| R+...)][ot*16+lr]
template <int NOT, bool RBF>
__device__ __forceinline__ void load_w_frag(const float* __restrict__ W, int R, int g, int f0,
                                            int lr, int lq, float (&wf)[NOT][4][2]) {
#pragma unroll
  for (int ot = 0; ot < NOT; ++ot) {
    const int o = ot * 16 + lr;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int fr = f0 + 4 * lq + r;
      const bool ok = o < g && fr < R;
      wf[ot][r][0] = ok ? W[(int64_t)fr * g + o] : 0.f;
      wf[ot][r][1] = (RBF && ok) ? W[(int64_t)(R + fr) * g + o] : 0.f;
    }
  }
}

// ------------------------------------------------------------------------- forward
template <bool SMALLD, int NOT, bool RBF>
__global__ __launch_bounds__(256) void k_step_fwd(const dgprf_plan_t pl, const StepDev sd,
                                                  const int layer) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const StepLds LD = step_lds(pl, layer);
  const int chain = blockIdx.z, rt = blockIdx.x, sl = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, lr = lane & 15, lq = lane >> 4;
  const int d = pl.d[layer], R = pl.n_rf[layer], g = pl.n_gp[layer], B = pl.batch;
  const int row0 = rt * TR;
  int64_t* ridx = reinterpret_cast<int64_t*>(smem);
  float* xs = smem + 32;
  float* red = smem + LD.red_off;
  const float* __restrict__ om = sd.omega + pl.omega_off[layer];
  const float* __restrict__ W = sd.theta + (int64_t)chain * pl.w_total + pl.w_off[layer];
  const int cpw = pl.cpw[layer];
  auto chunk_f0 = [&](int i) { return ((sl * cpw + i) * NW + wave) * 16; };

  // prefetch the first chunk's fragments (independent of the X tile)
  float omk[8], wf[NOT][4][2];
  if (SMALLD) load_om_frag(om, R, d, chunk_f0(0), lr, lq, omk);
  load_w_frag<NOT, RBF>(W, R, g, chunk_f0(0), lr, lq, wf);
  const float cl = sd.der[layer];

  if (needs_rows(pl, layer)) {
    fill_ridx(pl, sd, chain, row0, cur_step(sd), ridx);
    __syncthreads();
  }
  load_x_tile(pl, sd, layer, chain, row0, ridx, xs, LD.xst);
  __syncthreads();

  float xf[8];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) xf[ks] = (SMALLD && 4 * ks < d) ? xs[lr * LD.xst + 4 * ks + lq] : 0.f;

  f4 acc[NOT], acs[NOT];
#pragma unroll
  for (int ot = 0; ot < NOT; ++ot) acc[ot] = acs[ot] = f4zero();
  for (int i = 0; i < cpw; ++i) {
    const int f0 = chunk_f0(i);
    if (f0 >= R) break;
    const f4 at = a_tile<SMALLD, false>(om, R, d, f0, omk, xf, xs, LD.xst, lr, lq);
    float p0[4], p1[4];
    features<RBF>(at, cl, p0, p1);
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        acc[ot] = mfma16(wf[ot][r][0], p0[r], acc[ot]);
        if (RBF) acs[ot] = mfma16(wf[ot][r][1], p1[r], acs[ot]);
      }
    if (i + 1 < cpw && chunk_f0(i + 1) < R) {
      if (SMALLD) load_om_frag(om, R, d, chunk_f0(i + 1), lr, lq, omk);
      load_w_frag<NOT, RBF>(W, R, g, chunk_f0(i + 1), lr, lq, wf);
    }
  }
  // acc[ot][r] = F[row lr][ot*16 + 4lq + r]; sum the 4 waves' feature chunks in LDS.
  constexpr int GP = NOT * 16;
  float* redw = red + wave * TR * GP;
#pragma unroll
  for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
    for (int r = 0; r < 4; ++r) redw[lr * GP + ot * 16 + 4 * lq + r] = acc[ot][r] + acs[ot][r];
  __syncthreads();
  float* fp = sd.ws + (int64_t)chain * pl.ws_chain + pl.fp_off[layer] + (int64_t)sl * B * g;
  for (int e = threadIdx.x; e < TR * g; e += blockDim.x) {
    const int r = e / g, o = e - r * g, b = row0 + r;
    if (b < B) {
      float v = red[r * GP + o];
#pragma unroll
      for (int w = 1; w < NW; ++w) v += red[w * TR * GP + r * GP + o];
      fp[(int64_t)b * g + o] = v;
    }
  }
}

// ------------------------------------------------------------------------- backward
template <bool SMALLD, int NOT, bool RBF>
__global__ __launch_bounds__(256) void k_step_bwd(const dgprf_plan_t pl, const StepDev sd,
                                                  const int layer) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const StepLds LD = step_lds(pl, layer);
  const int chain = blockIdx.z, rt = blockIdx.x, sl = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, lr = lane & 15, lq = lane >> 4;
  const int L = pl.n_layers;
  const int d = pl.d[layer], R = pl.n_rf[layer], g = pl.n_gp[layer], B = pl.batch;
  const int row0 = rt * TR;
  int64_t* ridx = reinterpret_cast<int64_t*>(smem);
  float* xs = smem + 32;
  float* dfs = smem + LD.aux_off;
  const int dfst = LD.auxst;
  float* red = smem + LD.red_off;
  float* wsc = sd.ws + (int64_t)chain * pl.ws_chain;
  const float* __restrict__ om = sd.omega + pl.omega_off[layer];
  const float* __restrict__ W = sd.theta + (int64_t)chain * pl.w_total + pl.w_off[layer];
  const int cpw = pl.cpw[layer];
  auto chunk_f0 = [&](int i) { return ((sl * cpw + i) * NW + wave) * 16; };
  const bool last = layer == L - 1;

  float omk[8];
  if (SMALLD) load_om_frag(om, R, d, chunk_f0(0), lr, lq, omk);
  const float cl = sd.der[layer];

  if (needs_rows(pl, layer) || last) {
    fill_ridx(pl, sd, chain, row0, cur_step(sd), ridx);
    __syncthreads();
  }
  load_x_tile(pl, sd, layer, chain, row0, ridx, xs, LD.xst);

  // dF_l tile [16][g]
  if (last) {
    // likelihood gradient dF = -(1/B) dlogp/dF (likelihoods/gaussian.py:18-25, softmax.py:8-15)
    const float* fpl = wsc + pl.fp_off[layer];
    const int64_t ss = (int64_t)B * g;
    for (int e = threadIdx.x; e < TR * g; e += blockDim.x) {  // F_L = sum of slices
      const int r = e / g, o = e - r * g, b = row0 + r;
      dfs[r * dfst + o] = b < B ? sum_slices(fpl + (int64_t)b * g + o, ss) : 0.f;
    }
    __syncthreads();
    if (threadIdx.x < TR) {
      const int r = threadIdx.x, b = row0 + r;
      float* df = dfs + r * dfst;
      if (b < B) {
        const float* y = sd.bd.Y + ridx[r] * sd.bd.y_cols;
        const float invB = 1.0f / (float)B;
        float logp = 0.f;
        if (pl.likelihood == DGPRF_LIK_GAUSSIAN) {
          const float var = sd.der[DGPRF_MAX_LAYERS];
          const float logvar = logf(var);
          for (int o = 0; o < g; ++o) {
            const float diff = y[o] - df[o];
            logp += -0.5f * (LOG_2PI + logvar + diff * diff / var);
            df[o] = -(diff / var) * invB;
          }
        } else {
          float mx = -INFINITY;
          for (int o = 0; o < g; ++o) mx = fmaxf(mx, df[o]);
          float se = 0.f;
          for (int o = 0; o < g; ++o) se += expf(df[o] - mx);
          const float lse = mx + logf(se);
          const int label = min(max((int)y[0], 0), g - 1);
          for (int o = 0; o < g; ++o) {
            const float f = df[o];
            if (o == label) logp = f - lse;
            df[o] = (expf(f - lse) - (o == label ? 1.f : 0.f)) * invB;
          }
        }
        if (sl == 0) wsc[pl.logp_off + b] = logp;
      } else {
        for (int o = 0; o < g; ++o) df[o] = 0.f;
      }
    }
  } else {
    // dF_l = dX_{l+1}[:, :g_l] summed over the slices of layer l+1
    const float* dx = wsc + pl.dxp_off[layer + 1];
    const int64_t ss = (int64_t)B * g;
    for (int e = threadIdx.x; e < TR * g; e += blockDim.x) {
      const int r = e / g, o = e - r * g, b = row0 + r;
      dfs[r * dfst + o] = b < B ? sum_slices(dx + (int64_t)b * g + o, ss) : 0.f;
    }
  }
  __syncthreads();

  const int KG = (g + 3) >> 2;
  const int dxw = layer > 0 ? pl.n_gp[layer - 1] : 0;
  const int ND = (dxw + 15) >> 4;

  float xf[8];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) xf[ks] = (SMALLD && 4 * ks < d) ? xs[lr * LD.xst + 4 * ks + lq] : 0.f;
  // dF fragments: dff[ks] = dF[row lr][4ks+lq]        (B operand of dPhi, K = g)
  //               dfg[ot][r] = dF[row 4lq+r][ot*16+lr] (B operand of gW, K = rows)
  float dff[4 * NOT];
#pragma unroll
  for (int ks = 0; ks < 4 * NOT; ++ks) {
    const int o = 4 * ks + lq;
    dff[ks] = (o < g) ? dfs[lr * dfst + o] : 0.f;
  }
  float dfg[NOT][4];
#pragma unroll
  for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int o = ot * 16 + lr;
      dfg[ot][r] = (o < g) ? dfs[(4 * lq + r) * dfst + o] : 0.f;
    }

  float* gwp = wsc + pl.gwp_off + (int64_t)rt * pl.w_total + pl.w_off[layer];
  f4 dxa[4] = {f4zero(), f4zero(), f4zero(), f4zero()};
  for (int i = 0; i < cpw; ++i) {
    const int f0 = chunk_f0(i);
    if (f0 >= R) break;
    if (i > 0 && SMALLD) load_om_frag(om, R, d, f0, lr, lq, omk);
    // ---- gW_l partial over this row tile: rows-in-registers orientation
    {
      const f4 at = a_tile<SMALLD, true>(om, R, d, f0, omk, xf, xs, LD.xst, lr, lq);
      float q0[4], q1[4];
      features<RBF>(at, cl, q0, q1);
#pragma unroll
      for (int ot = 0; ot < NOT; ++ot) {
        f4 gc = f4zero(), gs = f4zero();
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          gc = mfma16(q0[r], dfg[ot][r], gc);
          if (RBF) gs = mfma16(q1[r], dfg[ot][r], gs);
        }
        // gc[r] = gW[f0 + 4lq + r][ot*16 + lr]
        const int o = ot * 16 + lr;
        if (o < g) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int f = f0 + 4 * lq + r;
            if (f < R) {
              gwp[(int64_t)f * g + o] = gc[r];
              if (RBF) gwp[(int64_t)(R + f) * g + o] = gs[r];
            }
          }
        }
      }
    }
    if (layer > 0) {
      // ---- dPhi = dF W^T, dA, dX = dA Omega^T : features-in-registers orientation
      const f4 at = a_tile<SMALLD, false>(om, R, d, f0, omk, xf, xs, LD.xst, lr, lq);
      const int fa = f0 + lr;
      f4 dpc = f4zero(), dps = f4zero();
#pragma unroll
      for (int ks = 0; ks < 4 * NOT; ++ks) {
        if (ks < KG) {
          const int o = 4 * ks + lq;
          const bool ok = fa < R && o < g;
          const float wc = ok ? W[(int64_t)fa * g + o] : 0.f;
          dpc = mfma16(wc, dff[ks], dpc);
          if (RBF) {
            const float wsn = ok ? W[(int64_t)(R + fa) * g + o] : 0.f;
            dps = mfma16(wsn, dff[ks], dps);
          }
        }
      }
      float da[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (RBF) {
          float s, c;
          rf_sincos(at[r], &s, &c);
          da[r] = -(cl * s) * dpc[r] + (cl * c) * dps[r];
        } else {
          da[r] = at[r] > 0.f ? cl * dpc[r] : 0.f;
        }
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        if (dt < ND) {
          const int k = dt * 16 + lr;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int f = f0 + 4 * lq + r;
            const float o = (k < dxw && f < R) ? om[(int64_t)k * R + f] : 0.f;
            dxa[dt] = mfma16(o, da[r], dxa[dt]);
          }
        }
      }
    }
  }
  if (layer > 0) {
    // dxa[dt][r] = dX[row lr][dt*16 + 4lq + r]; sum the 4 waves in LDS, store the slice partial.
    const int DP = ND * 16;
    float* redw = red + wave * TR * DP;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
      if (dt < ND)
#pragma unroll
        for (int r = 0; r < 4; ++r) redw[lr * DP + dt * 16 + 4 * lq + r] = dxa[dt][r];
    __syncthreads();
    float* dxp = wsc + pl.dxp_off[layer] + (int64_t)sl * B * dxw;
    for (int e = threadIdx.x; e < TR * dxw; e += blockDim.x) {
      const int r = e / dxw, k = e - r * dxw, b = row0 + r;
      if (b < B) {
        float v = red[r * DP + k];
#pragma unroll
        for (int w = 1; w < NW; ++w) v += red[w * TR * DP + r * DP + k];
        dxp[(int64_t)b * dxw + k] = v;
      }
    }
  }
}

// ------------------------------------------------------------------------- update
__device__ __forceinline__ f4 ld4(const float* p) { return *reinterpret_cast<const f4*>(p); }
__device__ __forceinline__ void st4(float* p, f4 v) { *reinterpret_cast<f4*>(p) = v; }

// cyclical_step_rate (utils.py:49-73) with min_value = 0 as used by the drivers
// (experiments/utils_training.py:53-54): lr = lr0 * rate^2.
__device__ __forceinline__ float cyclical_rate(int64_t step_index, int64_t cycle) {
  const float frac = (float)((step_index - 1) % cycle) / (float)cycle;
  return 0.0f + (1.0f - 0.0f) * 0.5f * (cosf(3.14159265358979f * frac) + 1.0f);
}

__global__ __launch_bounds__(256) void k_step_update(const dgprf_plan_t pl, const StepDev sd,
                                                     const UpdateDev ud,
                                                     const float* __restrict__ grad_in) {
  const int chain = blockIdx.y;
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t e0 = 4 * q;
  if (e0 >= pl.w_total) return;
  int layer = -1;
  for (int l = 0; l < pl.n_layers; ++l)
    if (e0 >= pl.w_off[l] && e0 < pl.w_off[l] + (int64_t)pl.P[l] * pl.n_gp[l]) layer = l;
  if (layer < 0) return;
  const int64_t base = (int64_t)chain * pl.w_total + e0;
  const float N = ud.data_size;
  const f4 th = ld4(sd.theta + base);
  f4 gr;
  if (grad_in) {
    gr = ld4(grad_in + base);
  } else {
    // sum the row-tile gW partials: groups of 16 independent loads (padding rows are zero)
    const float* gp = sd.ws + (int64_t)chain * pl.ws_chain + pl.gwp_off + e0;
    f4 s = f4zero();
    for (int rt0 = 0; rt0 < pl.n_rt_pad; rt0 += 16) {
      f4 v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = ld4(gp + (int64_t)(rt0 + j) * pl.w_total);
#pragma unroll
      for (int j = 0; j < 16; ++j) s += v[j];
    }
    // dU/dW = W/N (prior N(0,1), models/dgp.py:129-136,171) + Phi^T dF (likelihood)
    gr = th / N + s;
  }
  if (ud.grad_only) {
    st4(sd.grad_out + base, gr);
    return;
  }
  const int64_t t = *sd.step + (int64_t)sd.step_offset;
  float lr = ud.lr, T = ud.temperature;
  int resample = ud.resample;
  if (ud.schedule == DGPRF_SCHED_CYCLICAL) {
    if (t < ud.start_step) {  // burn-in: fixed lr, zero temperature
      T = 0.f;
      resample = 0;
    } else {
      const int64_t si = t - ud.start_step + 1;
      const float rate = cyclical_rate(si, ud.cycle_length);
      lr = ud.lr * (rate * rate);
      T = 1.f;
      resample = ud.resample_head && (si % ud.cycle_length == 1);
    }
  }
  const float h = sqrtf(lr / N);
  const float M = sd.mass[chain * pl.n_layers + layer];
  const float beta = ud.beta;
  f4 m = ld4(sd.mom + base);
  const uint32_t quad = (uint32_t)(e0 >> 2);
  if (resample) {  // models/dgp.py:209-210 (ignores M, Appendix A.1)
    m = ud.xi_resample ? ld4(ud.xi_resample + base)
                       : philox_normal4(sd.seed, (uint64_t)t, DGPRF_RNG_RESAMPLE, chain, quad);
  }
  f4 mn = beta * m - (h * N) * gr;
  const f4 eps =
      ud.xi ? ld4(ud.xi + base) : philox_normal4(sd.seed, (uint64_t)t, DGPRF_RNG_NOISE, chain, quad);
  mn = mn + sqrtf(2.0f * (1.0f - beta) * T * M) * eps;
  st4(sd.mom + base, mn);
  st4(sd.theta + base, th + (h * (1.0f / M)) * mn);
}

__global__ void k_advance(int64_t* step, int64_t by) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *step += by;
}

#define DGPRF_STEP_LAUNCHER(NAME)                                                                  \
  template <bool S, int NOT>                                                                       \
  void NAME##_kind(bool rbf, dim3 grid, size_t lds, hipStream_t s, const dgprf_plan_t& pl,         \
                   const StepDev& sd, int layer) {                                                 \
    if (rbf) {                                                                                     \
      dgprf::set_lds_limit((const void*)k_##NAME<S, NOT, true>, lds);                              \
      hipLaunchKernelGGL((k_##NAME<S, NOT, true>), grid, dim3(256), lds, s, pl, sd, layer);        \
    } else {                                                                                       \
      dgprf::set_lds_limit((const void*)k_##NAME<S, NOT, false>, lds);                             \
      hipLaunchKernelGGL((k_##NAME<S, NOT, false>), grid, dim3(256), lds, s, pl, sd, layer);       \
    }                                                                                              \
  }                                                                                                \
  template <bool S>                                                                                \
  void NAME##_not(int NOT, bool rbf, dim3 grid, size_t lds, hipStream_t s, const dgprf_plan_t& pl, \
                  const StepDev& sd, int layer) {                                                  \
    switch (NOT) {                                                                                 \
      case 1: NAME##_kind<S, 1>(rbf, grid, lds, s, pl, sd, layer); break;                          \
      case 2: NAME##_kind<S, 2>(rbf, grid, lds, s, pl, sd, layer); break;                          \
      case 3: NAME##_kind<S, 3>(rbf, grid, lds, s, pl, sd, layer); break;                          \
      default: NAME##_kind<S, 4>(rbf, grid, lds, s, pl, sd, layer); break;                         \
    }                                                                                              \
  }

DGPRF_STEP_LAUNCHER(step_fwd)
DGPRF_STEP_LAUNCHER(step_bwd)

}  // namespace

namespace dgprf {

static inline bool small_d(const dgprf_plan_t& pl, int layer) { return pl.d[layer] <= 32; }

hipError_t launch_step_fwd(const dgprf_plan_t& pl, const StepDev& sd, int layer, hipStream_t s) {
  const StepLds LD = step_lds(pl, layer);
  dim3 grid(pl.n_row_tiles, pl.ns[layer], pl.n_chains);
  const size_t lds = (size_t)LD.total * sizeof(float);
  const int NOT = (pl.n_gp[layer] + 15) >> 4;
  const bool rbf = pl.kind[layer] == DGPRF_RBF;
  if (small_d(pl, layer))
    step_fwd_not<true>(NOT, rbf, grid, lds, s, pl, sd, layer);
  else
    step_fwd_not<false>(NOT, rbf, grid, lds, s, pl, sd, layer);
  return hipGetLastError();
}

hipError_t launch_step_bwd(const dgprf_plan_t& pl, const StepDev& sd, int layer, hipStream_t s) {
  const StepLds LD = step_lds(pl, layer);
  dim3 grid(pl.n_row_tiles, pl.ns[layer], pl.n_chains);
  const size_t lds = (size_t)LD.total * sizeof(float);
  const int NOT = (pl.n_gp[layer] + 15) >> 4;
  const bool rbf = pl.kind[layer] == DGPRF_RBF;
  if (small_d(pl, layer))
    step_bwd_not<true>(NOT, rbf, grid, lds, s, pl, sd, layer);
  else
    step_bwd_not<false>(NOT, rbf, grid, lds, s, pl, sd, layer);
  return hipGetLastError();
}

hipError_t launch_step_update(const dgprf_plan_t& pl, const StepDev& sd, const UpdateDev& ud,
                              const float* grad_in, hipStream_t s) {
  const int64_t quads = pl.w_total / 4;
  dim3 grid((unsigned)((quads + 255) / 256), pl.n_chains);
  hipLaunchKernelGGL(k_step_update, grid, dim3(256), 0, s, pl, sd, ud, grad_in);
  return hipGetLastError();
}

hipError_t launch_advance(int64_t* step, int64_t by, hipStream_t s) {
  hipLaunchKernelGGL(k_advance, dim3(1), dim3(64), 0, s, step, by);
  return hipGetLastError();
}

}  // namespace dgprf
