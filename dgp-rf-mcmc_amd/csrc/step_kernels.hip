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
//   the SGHMC update with Philox noise.
//
// Latency discipline (this path is latency-bound): every kernel gets a compact
// host-precomputed argument block (one round of independent scalar loads, no plan indexing);
// fragment loads are unconditional with clamped addresses (no exec-masked branches or per-load
// waits) and are issued before the dependent partial sums; minibatch rows of step t+1 are gathered
// by step t's update kernel, so the forward never waits on the step counter or the permutation.
#include "dgprf_internal.h"

namespace {

constexpr int NW = DGPRF_WAVES;
constexpr int TR = DGPRF_TILE_ROWS;
constexpr int NSM = DGPRF_NS_MAX;
constexpr float LOG_2PI = 1.8378770664093453f;

__host__ __device__ __forceinline__ int round4(int x) { return (x + 3) & ~3; }

// Arguments of one forward / backward launch of layer `layer` (host-precomputed).
struct LayerK {
  const float* om;      // Omega_l [d][R]
  const float* W;       // W_l [P][g] of chain 0 (chain stride w_cs)
  const float* fprev;   // F_{l-1} partials [NSM][B][gp] of chain 0 (chain stride ws_cs)
  float* fout;          // F_l partials [NSM][B][g]
  const float* dxnext;  // dX_{l+1} partials [NSM][B][g]        (backward, l < L-1)
  float* dxout;         // dX_l partials [NSM][B][dxw]           (backward, l > 0)
  float* gwp;           // gW partials of W_l, row-tile stride w_cs (backward)
  float* logp;          // per-row log p [B]                       (backward, last layer)
  const float* xrows;   // minibatch X rows [B][d_in] (chain stride xrow_cs)
  const float* yrows;   // minibatch Y rows [B][y_cols] (chain stride yrow_cs)
  const float* cptr;    // c_l
  const float* varptr;  // sigma^2
  int64_t w_cs, ws_cs, xrow_cs, yrow_cs;
  int32_t d, R, g, gp, dxw, cpw, B, d_in, y_cols;
  int32_t last, likelihood, layer;
  int32_t xst, aux_off, auxst, red_off;
};

// Arguments of the update kernel.
struct UpdK {
  float* theta;
  float* mom;
  const float* mass;
  const float* gwp;     // gW partials base of chain 0 (chain stride ws_cs, row-tile stride w_total)
  const float* grad_in;
  float* grad_out;
  const int64_t* step;
  uint64_t seed;
  int64_t w_total, ws_cs;
  int64_t lo[DGPRF_MAX_LAYERS], hi[DGPRF_MAX_LAYERS];
  int32_t n_rt_pad, n_layers, step_offset, upd_blocks;
  UpdateDev ud;
  // gather of step t+1's minibatch rows (graph mode)
  int32_t gather_next, B, d_in, yb_cols;
  BatchDev bd;
  float* xb;
  float* yb;
};

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

__host__ __device__ inline void step_lds(int d, int g, LayerK& a, int& total) {
  a.xst = round4(d) + 1;
  a.aux_off = round4(TR * a.xst);
  a.auxst = g + 1;
  a.red_off = a.aux_off + 2 * round4(TR * a.auxst);  // dF tile + Y tile
  total = a.red_off + NW * TR * 64;
}

// X_l[16][d] of batch rows row0..: F_{l-1} partial sums (+ [F | X] dataset columns for input_cat,
// utils.py:42) or the gathered minibatch rows for layer 0.
__device__ __forceinline__ void load_x_tile(const LayerK& a, int chain, int row0, float* xs) {
  const int dpad = round4(a.d);
  const float* fprev = a.fprev + (int64_t)chain * a.ws_cs;
  const float* xr = a.xrows + (int64_t)chain * a.xrow_cs;
  for (int e = threadIdx.x; e < TR * dpad; e += blockDim.x) {
    const int r = e / dpad, k = e - r * dpad, b = row0 + r;
    const int bc = min(b, a.B - 1), kc = min(k, a.d - 1);
    float v;
    if (kc < a.gp)
      v = sum_slices(fprev + (int64_t)bc * a.gp + kc, (int64_t)a.B * a.gp);
    else
      v = xr[(int64_t)bc * a.d_in + (kc - a.gp)];
    xs[r * a.xst + k] = (b < a.B && k < a.d) ? v : 0.f;
  }
}

// Omega fragments: omk[ks] = Omega[4ks+lq][f0+lr] (zero outside the layer), KS k-steps.
template <int KS>
__device__ __forceinline__ void load_om_frag(const float* __restrict__ om, int R, int d, int f0,
                                             int lr, int lq, float (&omk)[8]) {
  const int fa = f0 + lr;
  const int fc = min(fa, R - 1);
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int k = 4 * ks + lq;
    const float v = om[(int64_t)min(k, d - 1) * R + fc];
    omk[ks] = (fa < R && k < d) ? v : 0.f;
  }
}

// A-tile.  TRANS=false: at[r] = A[row lr][f0+4lq+r] (features in regs)
//          TRANS=true : at[r] = A[row 4lq+r][f0+lr] (rows in regs)
template <int KS, bool TRANS>
__device__ __forceinline__ f4 a_tile(const float* __restrict__ om, int R, int d, int f0,
                                     const float (&omk)[8], const float (&xf)[8],
                                     const float* xs, int xst, int lr, int lq) {
  f4 at = f4zero();
  if (KS > 0) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      at = TRANS ? mfma16(xf[ks], omk[ks], at) : mfma16(omk[ks], xf[ks], at);
  } else {
    const int fa = f0 + lr, fc = min(fa, R - 1);
    const int nks = round4(d) >> 2;
    for (int ks = 0; ks < nks; ++ks) {
      const int k = 4 * ks + lq;
      const float ov = om[(int64_t)min(k, d - 1) * R + fc];
      const float o = (fa < R && k < d) ? ov : 0.f;
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

// Omega[k][f] with both indices clamped into the [rows][R] block (always a valid address).
__device__ __forceinline__ float om_safe(const float* __restrict__ om, int R, int rows, int k,
                                         int f) {
  return om[(int64_t)min(k, rows - 1) * R + min(f, R - 1)];
}

// W fragments for F^T += W^T Phi^T: wf[ot][r][0|1] = W[f0+4lq+r (| R+...)][ot*16+lr]
template <int NOT, bool RBF>
__device__ __forceinline__ void load_w_frag(const float* __restrict__ W, int R, int g, int f0,
                                            int lr, int lq, float (&wf)[NOT][4][2]) {
#pragma unroll
  for (int ot = 0; ot < NOT; ++ot) {
    const int o = ot * 16 + lr, oc = min(o, g - 1);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int fr = f0 + 4 * lq + r, fc = min(fr, R - 1);
      const bool ok = o < g && fr < R;
      const float v0 = W[(int64_t)fc * g + oc];
      wf[ot][r][0] = ok ? v0 : 0.f;
      if (RBF) {
        const float v1 = W[(int64_t)(R + fc) * g + oc];
        wf[ot][r][1] = ok ? v1 : 0.f;
      } else {
        wf[ot][r][1] = 0.f;
      }
    }
  }
}

// ------------------------------------------------------------------------- forward
template <int KS, int NOT, bool RBF>
__global__ __launch_bounds__(256) void k_step_fwd(const LayerK a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int chain = blockIdx.z, rt = blockIdx.x, sl = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, lr = lane & 15, lq = lane >> 4;
  const int R = a.R, g = a.g, d = a.d, B = a.B, cpw = a.cpw;
  const int row0 = rt * TR;
  const int stamp_base = (a.layer * 2) * 4096 + (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
  DGPRF_STAMP(stamp_base, 0);
  float* xs = smem;
  float* red = smem + a.red_off;
  const float* __restrict__ W = a.W + (int64_t)chain * a.w_cs;
  auto chunk_f0 = [&](int i) { return ((sl * cpw + i) * NW + wave) * 16; };

  // first chunk's fragments: independent of the X tile, issued first
  float omk[8], wf[NOT][4][2];
  if (KS > 0) load_om_frag<KS>(a.om, R, d, chunk_f0(0), lr, lq, omk);
  load_w_frag<NOT, RBF>(W, R, g, chunk_f0(0), lr, lq, wf);
  const float cl = *a.cptr;
  DGPRF_STAMP(stamp_base, 1);
  load_x_tile(a, chain, row0, xs);
  __syncthreads();
  DGPRF_STAMP(stamp_base, 2);

  float xf[8];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) xf[ks] = (ks < KS && 4 * ks < d) ? xs[lr * a.xst + 4 * ks + lq] : 0.f;

  f4 acc[NOT], acs[NOT];
#pragma unroll
  for (int ot = 0; ot < NOT; ++ot) acc[ot] = acs[ot] = f4zero();
  for (int i = 0; i < cpw; ++i) {
    const int f0 = chunk_f0(i);
    if (f0 >= R) break;
    const f4 at = a_tile<KS, false>(a.om, R, d, f0, omk, xf, xs, a.xst, lr, lq);
    float p0[4], p1[4];
    features<RBF>(at, cl, p0, p1);
    float wc[NOT][4][2];
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        wc[ot][r][0] = wf[ot][r][0];
        wc[ot][r][1] = wf[ot][r][1];
      }
    if (i + 1 < cpw) {  // prefetch the next chunk (clamped loads are always in range)
      if (KS > 0) load_om_frag<KS>(a.om, R, d, chunk_f0(i + 1), lr, lq, omk);
      load_w_frag<NOT, RBF>(W, R, g, chunk_f0(i + 1), lr, lq, wf);
    }
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        acc[ot] = mfma16(wc[ot][r][0], p0[r], acc[ot]);
        if (RBF) acs[ot] = mfma16(wc[ot][r][1], p1[r], acs[ot]);
      }
  }
  // acc[ot][r] = F[row lr][ot*16 + 4lq + r]; sum the 4 waves' feature chunks in LDS.
  constexpr int GP = NOT * 16;
  float* redw = red + wave * TR * GP;
#pragma unroll
  for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
    for (int r = 0; r < 4; ++r) redw[lr * GP + ot * 16 + 4 * lq + r] = acc[ot][r] + acs[ot][r];
  DGPRF_STAMP(stamp_base, 3);
  __syncthreads();
  float* fp = a.fout + (int64_t)chain * a.ws_cs + (int64_t)sl * B * g;
  for (int e = threadIdx.x; e < TR * g; e += blockDim.x) {
    const int r = e / g, o = e - r * g, b = row0 + r;
    if (b < B) {
      float v = red[r * GP + o];
#pragma unroll
      for (int w = 1; w < NW; ++w) v += red[w * TR * GP + r * GP + o];
      fp[(int64_t)b * g + o] = v;
    }
  }
#ifdef DGPRF_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  DGPRF_STAMP(stamp_base, 14);
}

// ------------------------------------------------------------------------- backward
template <int KS, int NOT, bool RBF>
__global__ __launch_bounds__(256) void k_step_bwd(const LayerK a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int chain = blockIdx.z, rt = blockIdx.x, sl = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, lr = lane & 15, lq = lane >> 4;
  const int R = a.R, g = a.g, d = a.d, B = a.B, cpw = a.cpw, dxw = a.dxw;
  const int row0 = rt * TR;
  const int stamp_base = (a.layer * 2 + 1) * 4096 + (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
  DGPRF_STAMP(stamp_base, 0);
  float* xs = smem;
  float* dfs = smem + a.aux_off;
  const int dfst = a.auxst;
  float* red = smem + a.red_off;
  const float* __restrict__ W = a.W + (int64_t)chain * a.w_cs;
  auto chunk_f0 = [&](int i) { return ((sl * cpw + i) * NW + wave) * 16; };
  constexpr int KGM = 4 * NOT;  // k-steps of the dPhi contraction (K = g)
  const int ND = (dxw + 15) >> 4;

  // first chunk's fragments, issued before the dependent partial sums
  float omk[8];
  if (KS > 0) load_om_frag<KS>(a.om, R, d, chunk_f0(0), lr, lq, omk);
  float wdp[KGM][2];  // dPhi A operand: W[f0+lr (| R+...)][4ks+lq]
  float omx[4][4];    // dX A operand: Omega[dt*16+lr][f0+4lq+r]
  auto load_bwd_frag = [&](int f0) {
    const int fa = f0 + lr, fc = min(fa, R - 1);
#pragma unroll
    for (int ks = 0; ks < KGM; ++ks) {
      const int o = 4 * ks + lq, oc = min(o, g - 1);
      const bool ok = fa < R && o < g;
      const float v0 = W[(int64_t)fc * g + oc];
      wdp[ks][0] = ok ? v0 : 0.f;
      if (RBF) {
        const float v1 = W[(int64_t)(R + fc) * g + oc];
        wdp[ks][1] = ok ? v1 : 0.f;
      } else {
        wdp[ks][1] = 0.f;
      }
    }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = dt * 16 + lr, f = f0 + 4 * lq + r;
        const float v = om_safe(a.om, R, max(dxw, 1), k, f);
        omx[dt][r] = (k < dxw && f < R) ? v : 0.f;
      }
  };
  if (dxw > 0) load_bwd_frag(chunk_f0(0));
  const float cl = *a.cptr;
  load_x_tile(a, chain, row0, xs);

  // dF_l tile [16][g]
  if (a.last) {
    // likelihood gradient dF = -(1/B) dlogp/dF (likelihoods/gaussian.py:18-25, softmax.py:8-15)
    const float* fpl = a.fout + (int64_t)chain * a.ws_cs;
    const float* yr = a.yrows + (int64_t)chain * a.yrow_cs;
    float* ysh = dfs + round4(TR * dfst);
    const int yc = a.likelihood == DGPRF_LIK_GAUSSIAN ? g : 1;
    for (int e = threadIdx.x; e < TR * g; e += blockDim.x) {  // F_L = sum of slices; Y alongside
      const int r = e / g, o = e - r * g, b = row0 + r, bc = min(b, B - 1);
      const float v = sum_slices(fpl + (int64_t)bc * g + o, (int64_t)B * g);
      const float yv = yr[(int64_t)bc * a.y_cols + min(o, yc - 1)];
      dfs[r * dfst + o] = b < B ? v : 0.f;
      ysh[r * dfst + o] = yv;
    }
    __syncthreads();
    if (threadIdx.x < TR) {
      const int r = threadIdx.x, b = row0 + r;
      float* df = dfs + r * dfst;
      if (b < B) {
        const float* y = ysh + r * dfst;
        const float invB = 1.0f / (float)B;
        float logp = 0.f;
        if (a.likelihood == DGPRF_LIK_GAUSSIAN) {
          const float var = *a.varptr;
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
        if (sl == 0) a.logp[(int64_t)chain * a.ws_cs + b] = logp;
      }
    }
  } else {
    // dF_l = dX_{l+1}[:, :g_l] summed over the slices of layer l+1
    const float* dx = a.dxnext + (int64_t)chain * a.ws_cs;
    for (int e = threadIdx.x; e < TR * g; e += blockDim.x) {
      const int r = e / g, o = e - r * g, b = row0 + r;
      const float v = sum_slices(dx + (int64_t)min(b, B - 1) * g + o, (int64_t)B * g);
      dfs[r * dfst + o] = b < B ? v : 0.f;
    }
  }
  __syncthreads();
  DGPRF_STAMP(stamp_base, 2);

  float xf[8];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) xf[ks] = (ks < KS && 4 * ks < d) ? xs[lr * a.xst + 4 * ks + lq] : 0.f;
  // dF fragments: dff[ks] = dF[row lr][4ks+lq]        (B operand of dPhi, K = g)
  //               dfg[ot][r] = dF[row 4lq+r][ot*16+lr] (B operand of gW, K = rows)
  float dff[KGM];
#pragma unroll
  for (int ks = 0; ks < KGM; ++ks) {
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
  const int KG = (g + 3) >> 2;

  float* gwp = a.gwp + (int64_t)chain * a.ws_cs + (int64_t)rt * a.w_cs;
  f4 dxa[4] = {f4zero(), f4zero(), f4zero(), f4zero()};
  for (int i = 0; i < cpw; ++i) {
    const int f0 = chunk_f0(i);
    if (f0 >= R) break;
    if (i > 0) {
      if (KS > 0) load_om_frag<KS>(a.om, R, d, f0, lr, lq, omk);
      if (dxw > 0) load_bwd_frag(f0);
    }
    // ---- gW_l partial over this row tile: rows-in-registers orientation
    {
      const f4 at = a_tile<KS, true>(a.om, R, d, f0, omk, xf, xs, a.xst, lr, lq);
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
    if (dxw > 0) {
      // ---- dPhi = dF W^T, dA, dX = dA Omega^T : features-in-registers orientation
      const f4 at = a_tile<KS, false>(a.om, R, d, f0, omk, xf, xs, a.xst, lr, lq);
      f4 dpc = f4zero(), dps = f4zero();
#pragma unroll
      for (int ks = 0; ks < KGM; ++ks) {
        if (ks < KG) {
          dpc = mfma16(wdp[ks][0], dff[ks], dpc);
          if (RBF) dps = mfma16(wdp[ks][1], dff[ks], dps);
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
      for (int dt = 0; dt < 4; ++dt)
        if (dt < ND)
#pragma unroll
          for (int r = 0; r < 4; ++r) dxa[dt] = mfma16(omx[dt][r], da[r], dxa[dt]);
    }
  }
  DGPRF_STAMP(stamp_base, 3);
  if (dxw > 0) {
    // dxa[dt][r] = dX[row lr][dt*16 + 4lq + r]; sum the 4 waves in LDS, store the slice partial.
    const int DP = ND * 16;
    float* redw = red + wave * TR * DP;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
      if (dt < ND)
#pragma unroll
        for (int r = 0; r < 4; ++r) redw[lr * DP + dt * 16 + 4 * lq + r] = dxa[dt][r];
    __syncthreads();
    float* dxp = a.dxout + (int64_t)chain * a.ws_cs + (int64_t)sl * B * dxw;
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
#ifdef DGPRF_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  DGPRF_STAMP(stamp_base, 14);
}

// ------------------------------------------------------------------------- update / gather
__device__ __forceinline__ f4 ld4(const float* p) { return *reinterpret_cast<const f4*>(p); }
__device__ __forceinline__ void st4(float* p, f4 v) { *reinterpret_cast<f4*>(p) = v; }

// cyclical_step_rate (utils.py:49-73) with min_value = 0 as used by the drivers
// (experiments/utils_training.py:53-54): lr = lr0 * rate^2.
__device__ __forceinline__ float cyclical_rate(int64_t step_index, int64_t cycle) {
  const float frac = (float)((step_index - 1) % cycle) / (float)cycle;
  return 0.0f + (1.0f - 0.0f) * 0.5f * (cosf(3.14159265358979f * frac) + 1.0f);
}

// Copy minibatch row b of chain `chain` at step t into the gathered-rows workspace.
__device__ __forceinline__ void gather_row(const BatchDev& bd, int B, int d_in, int yb_cols,
                                           float* xb, float* yb, int chain, int64_t t, int b) {
  const int64_t row = batch_row(bd, B, chain, t, b);
  const float* xs = bd.X + row * d_in;
  const float* ys = bd.Y + row * bd.y_cols;
  float* xd = xb + (int64_t)b * d_in;
  float* yd = yb + (int64_t)b * yb_cols;
  for (int k = 0; k < d_in; ++k) xd[k] = xs[k];
  for (int k = 0; k < yb_cols; ++k) yd[k] = ys[k];
}

struct GatherK {
  BatchDev bd;
  const int64_t* step;
  float* xb;  // chain 0 (chain stride ws_cs)
  float* yb;
  int64_t ws_cs;
  int32_t B, d_in, yb_cols, step_offset;
};

__global__ void k_gather(const GatherK a) {
  const int chain = blockIdx.y;
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= a.B) return;
  const int64_t t = *a.step + a.step_offset;
  gather_row(a.bd, a.B, a.d_in, a.yb_cols, a.xb + (int64_t)chain * a.ws_cs,
             a.yb + (int64_t)chain * a.ws_cs, chain, t, b);
}

__global__ __launch_bounds__(256) void k_step_update(const UpdK a) {
  const int chain = blockIdx.y;
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t e0 = 4 * q;
  const int stamp_base = 16 * 4096 + blockIdx.y * gridDim.x + blockIdx.x;
  DGPRF_STAMP(stamp_base, 0);
  const UpdateDev& ud = a.ud;
  const int64_t t = *a.step + (int64_t)a.step_offset;
  if ((int)blockIdx.x >= a.upd_blocks) {  // dedicated blocks: rows of step t+1 (off the path)
    const int b = ((int)blockIdx.x - a.upd_blocks) * blockDim.x + threadIdx.x;
    if (a.gather_next && b < a.B)
      gather_row(a.bd, a.B, a.d_in, a.yb_cols, a.xb + (int64_t)chain * a.ws_cs,
                 a.yb + (int64_t)chain * a.ws_cs, chain, t + 1, b);
    return;
  }
  if (e0 >= a.w_total) return;
  int layer = -1;
#pragma unroll
  for (int l = 0; l < DGPRF_MAX_LAYERS; ++l)
    if (l < a.n_layers && e0 >= a.lo[l] && e0 < a.hi[l]) layer = l;
  if (layer < 0) return;
  const int64_t base = (int64_t)chain * a.w_total + e0;
  const float N = ud.data_size;
  const f4 th = ld4(a.theta + base);
  f4 gr;
  if (a.grad_in) {
    gr = ld4(a.grad_in + base);
  } else {
    // sum the row-tile gW partials: groups of 16 independent loads (padding rows are zero)
    const float* gp = a.gwp + (int64_t)chain * a.ws_cs + e0;
    f4 s = f4zero();
    for (int rt0 = 0; rt0 < a.n_rt_pad; rt0 += 16) {
      f4 v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = ld4(gp + (int64_t)(rt0 + j) * a.w_total);
#pragma unroll
      for (int j = 0; j < 16; ++j) s += v[j];
    }
    // dU/dW = W/N (prior N(0,1), models/dgp.py:129-136,171) + Phi^T dF (likelihood)
    gr = th / N + s;
  }
  if (ud.grad_only) {
    st4(a.grad_out + base, gr);
    return;
  }
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
  const float M = a.mass[chain * a.n_layers + layer];
  const float beta = ud.beta;
  f4 m = ld4(a.mom + base);
  const uint32_t quad = (uint32_t)(e0 >> 2);
  if (resample) {  // models/dgp.py:209-210 (ignores M, Appendix A.1)
    m = ud.xi_resample ? ld4(ud.xi_resample + base)
                       : philox_normal4(a.seed, (uint64_t)t, DGPRF_RNG_RESAMPLE, chain, quad);
  }
  f4 mn = beta * m - (h * N) * gr;
  const f4 eps =
      ud.xi ? ld4(ud.xi + base) : philox_normal4(a.seed, (uint64_t)t, DGPRF_RNG_NOISE, chain, quad);
  mn = mn + sqrtf(2.0f * (1.0f - beta) * T * M) * eps;
  st4(a.mom + base, mn);
  st4(a.theta + base, th + (h * (1.0f / M)) * mn);
#ifdef DGPRF_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  DGPRF_STAMP(stamp_base, 14);
}

__global__ void k_advance(int64_t* step, int64_t by) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *step += by;
}

// ------------------------------------------------------------------------- host helpers
LayerK make_layer_k(const dgprf_plan_t& pl, const StepDev& sd, int l, int& lds_floats) {
  LayerK a;
  const bool direct = sd.bd.mode == DGPRF_BATCH_DIRECT;
  a.om = sd.omega + pl.omega_off[l];
  a.W = sd.theta + pl.w_off[l];
  a.fprev = l > 0 ? sd.ws + pl.fp_off[l - 1] : sd.ws;
  a.fout = sd.ws + pl.fp_off[l];
  a.dxnext = l + 1 < pl.n_layers ? sd.ws + pl.dxp_off[l + 1] : sd.ws;
  a.dxout = l > 0 ? sd.ws + pl.dxp_off[l] : sd.ws;
  a.gwp = sd.ws + pl.gwp_off + pl.w_off[l];
  a.logp = sd.ws + pl.logp_off;
  a.xrows = direct ? sd.bd.X : sd.ws + pl.xb_off;
  a.yrows = direct ? sd.bd.Y : sd.ws + pl.yb_off;
  a.xrow_cs = direct ? 0 : pl.ws_chain;
  a.yrow_cs = direct ? 0 : pl.ws_chain;
  a.y_cols = direct ? sd.bd.y_cols : pl.yb_cols;
  a.cptr = sd.der + l;
  a.varptr = sd.der + DGPRF_MAX_LAYERS;
  a.w_cs = pl.w_total;
  a.ws_cs = pl.ws_chain;
  a.d = pl.d[l];
  a.R = pl.n_rf[l];
  a.g = pl.n_gp[l];
  a.gp = l > 0 ? pl.n_gp[l - 1] : 0;
  a.dxw = l > 0 ? pl.n_gp[l - 1] : 0;
  a.cpw = pl.cpw[l];
  a.B = pl.batch;
  a.d_in = pl.d_in;
  a.last = l == pl.n_layers - 1;
  a.likelihood = pl.likelihood;
  a.layer = l;
  step_lds(a.d, a.g, a, lds_floats);
  return a;
}

#define DGPRF_KS_NOT_DISPATCH(KERNEL)                                                              \
  template <int KS, int NOT>                                                                       \
  void KERNEL##_launch3(bool rbf, dim3 grid, size_t lds, hipStream_t s, const LayerK& a) {         \
    if (rbf) {                                                                                     \
      dgprf::set_lds_limit((const void*)KERNEL<KS, NOT, true>, lds);                               \
      hipLaunchKernelGGL((KERNEL<KS, NOT, true>), grid, dim3(256), lds, s, a);                     \
    } else {                                                                                       \
      dgprf::set_lds_limit((const void*)KERNEL<KS, NOT, false>, lds);                              \
      hipLaunchKernelGGL((KERNEL<KS, NOT, false>), grid, dim3(256), lds, s, a);                    \
    }                                                                                              \
  }                                                                                                \
  template <int KS>                                                                                \
  void KERNEL##_launch2(int NOT, bool rbf, dim3 grid, size_t lds, hipStream_t s,                   \
                        const LayerK& a) {                                                         \
    switch (NOT) {                                                                                 \
      case 1: KERNEL##_launch3<KS, 1>(rbf, grid, lds, s, a); break;                                \
      case 2: KERNEL##_launch3<KS, 2>(rbf, grid, lds, s, a); break;                                \
      case 3: KERNEL##_launch3<KS, 3>(rbf, grid, lds, s, a); break;                                \
      default: KERNEL##_launch3<KS, 4>(rbf, grid, lds, s, a); break;                               \
    }                                                                                              \
  }                                                                                                \
  void KERNEL##_launch(int d, int NOT, bool rbf, dim3 grid, size_t lds, hipStream_t s,             \
                       const LayerK& a) {                                                          \
    if (d <= 4) KERNEL##_launch2<1>(NOT, rbf, grid, lds, s, a);                                    \
    else if (d <= 8) KERNEL##_launch2<2>(NOT, rbf, grid, lds, s, a);                               \
    else if (d <= 16) KERNEL##_launch2<4>(NOT, rbf, grid, lds, s, a);                              \
    else if (d <= 32) KERNEL##_launch2<8>(NOT, rbf, grid, lds, s, a);                              \
    else KERNEL##_launch2<0>(NOT, rbf, grid, lds, s, a);                                           \
  }

DGPRF_KS_NOT_DISPATCH(k_step_fwd)
DGPRF_KS_NOT_DISPATCH(k_step_bwd)

}  // namespace

#ifdef DGPRF_STAMPS
__device__ unsigned long long g_dgprf_stamps[17 * 4096 * DGPRF_STAMP_SLOTS];
extern "C" int dgprf_debug_read_stamps(unsigned long long* host, long long n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_dgprf_stamps), (size_t)n * 8, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : -3;
}
extern "C" int dgprf_debug_clear_stamps(void) {
  static unsigned long long zeros[17 * 4096 * DGPRF_STAMP_SLOTS];
  return hipMemcpyToSymbol(HIP_SYMBOL(g_dgprf_stamps), zeros, sizeof(zeros), 0,
                           hipMemcpyHostToDevice) == hipSuccess ? 0 : -3;
}
#endif

namespace dgprf {

hipError_t launch_step_fwd(const dgprf_plan_t& pl, const StepDev& sd, int layer, hipStream_t s) {
  int lds_floats = 0;
  const LayerK a = make_layer_k(pl, sd, layer, lds_floats);
  dim3 grid(pl.n_row_tiles, pl.ns[layer], pl.n_chains);
  const int NOT = (pl.n_gp[layer] + 15) >> 4;
  k_step_fwd_launch(pl.d[layer], NOT, pl.kind[layer] == DGPRF_RBF, grid,
                    (size_t)lds_floats * sizeof(float), s, a);
  return hipGetLastError();
}

hipError_t launch_step_bwd(const dgprf_plan_t& pl, const StepDev& sd, int layer, hipStream_t s) {
  int lds_floats = 0;
  const LayerK a = make_layer_k(pl, sd, layer, lds_floats);
  dim3 grid(pl.n_row_tiles, pl.ns[layer], pl.n_chains);
  const int NOT = (pl.n_gp[layer] + 15) >> 4;
  k_step_bwd_launch(pl.d[layer], NOT, pl.kind[layer] == DGPRF_RBF, grid,
                    (size_t)lds_floats * sizeof(float), s, a);
  return hipGetLastError();
}

hipError_t launch_step_update(const dgprf_plan_t& pl, const StepDev& sd, const UpdateDev& ud,
                              const float* grad_in, hipStream_t s, bool gather_next) {
  UpdK a;
  a.theta = sd.theta;
  a.mom = sd.mom;
  a.mass = sd.mass;
  a.gwp = sd.ws ? sd.ws + pl.gwp_off : nullptr;
  a.grad_in = grad_in;
  a.grad_out = sd.grad_out;
  a.step = sd.step;
  a.seed = sd.seed;
  a.w_total = pl.w_total;
  a.ws_cs = pl.ws_chain;
  for (int l = 0; l < DGPRF_MAX_LAYERS; ++l) {
    a.lo[l] = l < pl.n_layers ? pl.w_off[l] : 0;
    a.hi[l] = l < pl.n_layers ? pl.w_off[l] + (int64_t)pl.P[l] * pl.n_gp[l] : 0;
  }
  a.n_rt_pad = pl.n_rt_pad;
  a.n_layers = pl.n_layers;
  a.step_offset = sd.step_offset;
  a.ud = ud;
  a.gather_next = gather_next && sd.bd.mode == DGPRF_BATCH_EPOCH ? 1 : 0;
  a.B = pl.batch;
  a.d_in = pl.d_in;
  a.yb_cols = pl.yb_cols;
  a.bd = sd.bd;
  a.xb = sd.ws ? sd.ws + pl.xb_off : nullptr;
  a.yb = sd.ws ? sd.ws + pl.yb_off : nullptr;
  const int64_t quads = pl.w_total / 4;
  a.upd_blocks = (int)((quads + 255) / 256);
  const int64_t blocks = a.upd_blocks + (a.gather_next ? (pl.batch + 255) / 256 : 0);
  dim3 grid((unsigned)blocks, pl.n_chains);
  hipLaunchKernelGGL(k_step_update, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_gather(const dgprf_plan_t& pl, const StepDev& sd, hipStream_t s) {
  if (sd.bd.mode == DGPRF_BATCH_DIRECT) return hipSuccess;
  GatherK a;
  a.bd = sd.bd;
  a.step = sd.step;
  a.xb = sd.ws + pl.xb_off;
  a.yb = sd.ws + pl.yb_off;
  a.ws_cs = pl.ws_chain;
  a.B = pl.batch;
  a.d_in = pl.d_in;
  a.yb_cols = pl.yb_cols;
  a.step_offset = sd.step_offset;
  dim3 grid((unsigned)((pl.batch + 255) / 256), pl.n_chains);
  hipLaunchKernelGGL(k_gather, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_advance(int64_t* step, int64_t by, hipStream_t s) {
  hipLaunchKernelGGL(k_advance, dim3(1), dim3(64), 0, s, step, by);
  return hipGetLastError();
}

}  // namespace dgprf
