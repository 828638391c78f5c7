// step_bwdrg_impl.h — the row-group step backward k_step_bwd_rg for minibatches of more than 16 row
// tiles (B > 256), included by step_bwdrg_k<KS>.hip.
//
// Same arithmetic as k_step_bwd (the analytic form of tape.gradient, models/dgp.py:194-198, for one
// layer: likelihood gradient, gW_l = Phi_l^T dF_l, dPhi = dF W^T, dA, dX_l = dA Omega^T), but one
// workgroup owns a GROUP of rt_per_rg consecutive 16-row tiles x one feature slice and keeps the
// slice's gW in MFMA accumulators across the whole group, so the backward writes one gW partial row
// per row group — at most 16 (plan.n_gw_rows), whatever B — instead of one per row tile
// (SURVEY.md §8d B-sweep; the update kernel sums them).  Per workgroup:
//   * 16 waves = ncw chunk-waves x nrw row-waves: an iteration covers nrw row tiles (a "super tile"
//     of 16 nrw rows), wave (cw, rw) computes the slice's chunks i ncw + cw on row tile rw;
//   * the slice's W rows and Omega rows are staged in LDS once;
//   * the next iteration's X / dF partial sums (16 slices each) are loaded into registers while the
//     current iteration computes (register prefetch), then stored to LDS;
//   * dX of every iteration is reduced over the chunk-waves in LDS and stored as the slice partial;
//   * at the end the row-waves' gW accumulators are summed in LDS in row-wave order and the group's
//     gW partial row is written.
// Every sum runs in a fixed order (row tiles of the group in sequence inside the accumulators, then
// row-waves 0..nrw-1): deterministic, no atomics.
#pragma once
#include "step_common.h"

namespace dgprf_sk {

constexpr int RG_WAVES = 16;

// In-kernel timestamps of the diagnostic -DDGPRF_STAMPS build only (into the buffer the launcher
// passes in a.stamps; never in the product).
#ifdef DGPRF_STAMPS
#define RG_STAMP(base, i)                                                        \
  do {                                                                           \
    if (threadIdx.x == 0 && a.stamps) {                                          \
      __builtin_amdgcn_sched_barrier(0);                                         \
      a.stamps[(size_t)(base) * 16 + (i)] = __builtin_amdgcn_s_memtime();        \
      __builtin_amdgcn_sched_barrier(0);                                         \
    }                                                                            \
  } while (0)
#else
#define RG_STAMP(base, i) \
  do {                    \
    (void)(base);         \
  } while (0)
#endif

// One prologue element of a super tile (rows row0 .. row0 + rows, valid below row_end): X tile
// elements first (rows x dpad, only when need_x), then dF tile elements (rows x g) with their Y.
__device__ __forceinline__ void rg_issue(const LayerK& a, int chain, int row0, int row_end, int rows,
                                         int nx, int u, Elem& e) {
  const rsrc_t rws = make_rsrc(a.ws + (int64_t)chain * a.ws_cs, a.ws_cs);
  const rsrc_t rx = make_rsrc(a.xrows + (int64_t)chain * a.xrow_cs, (int64_t)a.B * (a.d - a.gp));
  const rsrc_t ry = make_rsrc(a.yrows + (int64_t)chain * a.yrow_cs, (int64_t)a.B * a.y_cols);
  const int dpad = round4(a.d), ndat = a.d - a.gp;
  const bool isx = u < nx, isd = !isx && u < nx + rows * a.g;
  const int ud = u - nx;
  const int r = isx ? (u * a.xmag) >> 20 : (ud * a.dmag) >> 20;
  const int c = isx ? u - r * dpad : ud - r * a.g;
  const int b = row0 + r;
  const bool inb = b < row_end && (isx || isd);
  const bool fromp = inb && (isx ? c < a.gp : true);
  const int w = isx ? a.gp : a.g;
  const int base = (isx ? a.fprev_off : a.dsrc_off) + b * w + c;
  const int str = a.B * w;
  // complete sources (fused forward: F_{l-1}, and F_L for the last layer) hold slice 0 only
  const int nsl = (a.cmp && (isx || a.last)) ? 1 : NSM;
#pragma unroll
  for (int sl = 0; sl < NSM; ++sl)
    e.v[sl] = bload1(rws, fromp && sl < nsl ? (uint32_t)((base + sl * str) * 4) : DGPRF_OOB);
  const bool xdat = inb && isx && c >= a.gp && c < a.d;
  e.xd = bload1(rx, xdat ? (uint32_t)((b * ndat + (c - a.gp)) * 4) : DGPRF_OOB);
  const int yc = a.likelihood == DGPRF_LIK_GAUSSIAN ? a.g : 1;
  const bool ydat = inb && isd && a.last;
  e.y = bload1(ry, ydat ? (uint32_t)((b * a.y_cols + min(c, yc - 1)) * 4) : DGPRF_OOB);
  e.isx = isx;
  e.dst = isx ? r * a.xst + c : (isd ? r * a.auxst + c : -1);
}

__device__ __forceinline__ void rg_store(const Elem& e, float* xs, float* dfs, float* ysh) {
  if (e.dst < 0) return;
  float acc = e.v[0];
#pragma unroll
  for (int sl = 1; sl < NSM; ++sl) acc += e.v[sl];
  if (e.isx) {
    xs[e.dst] = acc + e.xd;  // exactly one of the two is non-zero-sourced
  } else {
    dfs[e.dst] = acc;
    ysh[e.dst] = e.y;
  }
}

// Generic prologue (super tiles too wide for two elements per thread): plain loops.
__device__ __forceinline__ void rg_load_generic(const LayerK& a, int chain, int row0, int row_end,
                                                int rows, bool need_x, float* xs, float* dfs,
                                                float* ysh) {
  const int dpad = round4(a.d);
  const float* fprev = a.fprev + (int64_t)chain * a.ws_cs;
  const float* xr = a.xrows + (int64_t)chain * a.xrow_cs;
  if (need_x)
    for (int e = threadIdx.x; e < rows * dpad; e += blockDim.x) {
      const int r = e / dpad, k = e - r * dpad, b = row0 + r;
      const int bc = min(b, a.B - 1), kc = min(k, a.d - 1);
      float v;
      if (kc < a.gp)
        v = a.cmp ? fprev[(int64_t)bc * a.gp + kc]
                  : sum_slices(fprev + (int64_t)bc * a.gp + kc, (int64_t)a.B * a.gp);
      else
        v = xr[(int64_t)bc * a.d_in + (kc - a.gp)];
      xs[r * a.xst + k] = (b < row_end && k < a.d) ? v : 0.f;
    }
  const float* src = (a.last ? a.fout : a.dxnext) + (int64_t)chain * a.ws_cs;
  const float* yr = a.yrows + (int64_t)chain * a.yrow_cs;
  const int g = a.g, yc = a.likelihood == DGPRF_LIK_GAUSSIAN ? g : 1;
  for (int e = threadIdx.x; e < rows * g; e += blockDim.x) {
    const int r = e / g, o = e - r * g, b = row0 + r, bc = min(b, a.B - 1);
    const float v = (a.cmp && a.last) ? src[(int64_t)bc * g + o]
                                      : sum_slices(src + (int64_t)bc * g + o, (int64_t)a.B * g);
    dfs[r * a.auxst + o] = b < row_end ? v : 0.f;
    if (a.last) ysh[r * a.auxst + o] = yr[(int64_t)bc * a.y_cols + min(o, yc - 1)];
  }
}

// NIT: chunk iterations per wave (ceil(4 cpw / ncw) <= NIT).
template <int KS, int NOT, bool RBF, bool G1, bool FB, int NIT>
__global__ __launch_bounds__(64 * RG_WAVES) void k_step_bwd_rg(const LayerK a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  int rg, sl;
  if (!tile_of_block(a, rg, sl)) return;
  const int stamp_base = (a.layer * 2 + 1) * 4096 + blockIdx.z * gridDim.x + blockIdx.x;
  RG_STAMP(stamp_base, 0);
  const int chain = blockIdx.z;
  const float* __restrict__ om = a.om + (int64_t)chain * a.om_cs;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, lr = lane & 15, lq = lane >> 4;
  const int R = a.R, g = a.g, d = a.d, B = a.B, dxw = a.dxw;
  const int ncw = a.ncw, nrw = a.nrw;
  const int cw = wave & (ncw - 1), rw = wave / ncw;
  const int CH = 4 * a.cpw;  // 16-feature chunks of the slice
  const int nf = 64 * a.cpw, fb0 = sl * nf;
  const int n_rt_all = (B + TR - 1) / TR;
  const int rt0 = rg * a.rt_per_rg;
  const int rt_end = min(rt0 + a.rt_per_rg, n_rt_all);
  const int row_end = min(rt_end * TR, B);
  const int rows = TR * nrw;
  const int n_iter = (rt_end - rt0 + nrw - 1) / nrw;
  constexpr int KGM = 4 * NOT;
  const int ND = (dxw + 15) >> 4, DP = ND * 16;
  const bool dphi = FB || dxw > 0;
  const bool need_x = KS > 0 || !a.a0 || FB;
  float* xs = smem;                       // [rows][xst]
  float* dfs = smem + a.aux_off;          // [rows][auxst]
  float* ysh = dfs + round4(rows * a.auxst);
  float* red = smem + a.red_off;          // [16 waves][TR][DP]
  float* wsa = smem + a.wsa_off;          // [RBF ? 2 : 1][nf][g]
  float* osa = smem + a.osa_off;          // [dxw][osa_st]
  const float cl = a.cptr[(int64_t)chain * a.der_cs];

  // ---- the slice's W rows (both halves) and Omega rows k < dxw, once (zero past R)
  if (dphi) {
    const float* W = a.W + (int64_t)chain * a.w_cs;
    const int nh = RBF ? 2 : 1, nwf = nf * g;
    if (((int64_t)R * g) % 4 == 0) {
      const int n4 = nwf / 4;
      for (int e = threadIdx.x; e < nh * n4; e += blockDim.x) {
        const int h = e >= n4, e2 = 4 * (e - h * n4);
        f4 v = f4zero();
        if (fb0 + (e2 + 3) / g < R) v = *reinterpret_cast<const f4*>(W + ((int64_t)h * R + fb0) * g + e2);
        *reinterpret_cast<f4*>(wsa + h * nwf + e2) = v;
      }
    } else {
      for (int e = threadIdx.x; e < nh * nwf; e += blockDim.x) {
        const int h = e >= nwf, e2 = e - h * nwf;
        wsa[e] = fb0 + e2 / g < R ? W[((int64_t)h * R + fb0) * g + e2] : 0.f;
      }
    }
    for (int e = threadIdx.x; e < dxw * nf; e += blockDim.x) {
      const int k = e / nf, c = e - k * nf;
      osa[k * a.osa_st + c] = fb0 + c < R ? om[(int64_t)k * R + fb0 + c] : 0.f;
    }
  }
  // ---- per-chunk Omega fragments (KS > 0) and z fragments (FB), loaded once
  auto chunk_f0 = [&](int i) { return (sl * CH + i * ncw + cw) * 16; };
  auto chunk_ok = [&](int i) { return i * ncw + cw < CH && chunk_f0(i) < R; };
  float omk[NIT][8];
#pragma unroll
  for (int i = 0; i < NIT; ++i)
    if (KS > 0) load_om_frag<KS>(om, R, d, min(chunk_f0(i), R - 1), lr, lq, omk[i]);
  constexpr int NZ = KS > 0 ? (4 * KS + 15) / 16 : 0;
  const rsrc_t rz = make_rsrc(a.z, FB ? (int64_t)d * R : 0);
  auto z_frag = [&](int f0, int dt) -> f4 {
    const int k = dt * 16 + lr;
    return bload4(rz, k < d && f0 + 4 * lq < R ? (uint32_t)(((int64_t)k * R + f0 + 4 * lq) * 4)
                                               : DGPRF_OOB);
  };
  f4 zpf[NIT][NZ > 0 ? NZ : 1];
  if (FB)
#pragma unroll
    for (int i = 0; i < NIT; ++i)
#pragma unroll
      for (int dt = 0; dt < NZ; ++dt) zpf[i][dt] = z_frag(chunk_f0(i), dt);

  // ---- accumulators over the whole row group
  f4 gacc[NIT][NOT][2];
  float g1c[NIT], g1s[NIT];
#pragma unroll
  for (int i = 0; i < NIT; ++i) {
    g1c[i] = g1s[i] = 0.f;
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot) gacc[i][ot][0] = gacc[i][ot][1] = f4zero();
  }
  const int hst = round4(2 * d + 1);
  float* hw = smem + a.hred_off + wave * hst;
  float ampl = 0.f, lvacc = 0.f;
  if (FB)
    for (int e = lane; e < hst; e += 64) hw[e] = 0.f;

  // ---- prologue of the first super tile
  const int nx = need_x ? rows * round4(d) : 0;
  const int total = nx + rows * g;
  const int t = threadIdx.x;
  const int wave0 = __builtin_amdgcn_readfirstlane(t & ~63);
  Elem e0;  // one prologue element per thread (rg_fast: total <= 1024)
  e0.dst = -1;
  if (a.rg_fast && wave0 < total) rg_issue(a, chain, rt0 * TR, row_end, rows, nx, t, e0);
  RG_STAMP(stamp_base, 1);
  float* dxp = a.dxout + (int64_t)chain * a.ws_cs + (int64_t)sl * B * dxw;
  const float* a0b = KS == 0 && a.a0 ? a.a0 + (int64_t)chain * a.ws_cs : nullptr;

  for (int it = 0; it < n_iter; ++it) {
    const int row0 = (rt0 + it * nrw) * TR;
    if (a.rg_fast) {
      if (wave0 < total) rg_store(e0, xs, dfs, ysh);
    } else {
      rg_load_generic(a, chain, row0, row_end, rows, need_x, xs, dfs, ysh);
    }
    __syncthreads();
    if (it == 0) RG_STAMP(stamp_base, 2);
    if (a.last) {
      // likelihood gradient dF = -(1/B) dlogp/dF (likelihoods/gaussian.py:18-25, softmax.py:8-15)
      float lvrow = 0.f;
      if (threadIdx.x < rows) {
        const int r = threadIdx.x, b = row0 + r;
        float* df = dfs + r * a.auxst;
        if (b < row_end) {
          const float* y = ysh + r * a.auxst;
          const float invB = 1.0f / (float)B;
          float logp = 0.f;
          if (a.likelihood == DGPRF_LIK_GAUSSIAN) {
            const float var = a.varptr[(int64_t)chain * a.der_cs];
            const float logvar = logf(var);
            float lv = 0.f;
            for (int o = 0; o < g; ++o) {
              const float diff = y[o] - df[o];
              logp += -0.5f * (LOG_2PI + logvar + diff * diff / var);
              df[o] = -(diff / var) * invB;
              lv += 0.5f * (1.f - diff * diff / var);
            }
            lvrow = lv * invB;
          } else {
            float mx = -INFINITY;
            for (int o = 0; o < g; ++o) mx = fmaxf(mx, df[o]);
            float se = 0.f;
            for (int o = 0; o < g; ++o) se += expf(df[o] - mx);
            const float lse = mx + logf(se);
            const int label = (int)y[0];
            const float bad = (label >= 0 && label < g) ? 0.f : __builtin_nanf("");
            for (int o = 0; o < g; ++o) {
              const float f = df[o];
              if (o == label) logp = f - lse;
              df[o] = (expf(f - lse) - (o == label ? 1.f : 0.f)) * invB + bad;
            }
            logp += bad;
          }
          if (sl == 0) a.logp[(int64_t)chain * a.ws_cs + b] = logp;
        }
      }
      if (FB && a.lik_fb && wave == 0) {  // the super tile's lik_log_var term (fixed order)
        float v = sum16(lvrow);
        v += __shfl_xor(v, 16);
        v += __shfl_xor(v, 32);
        lvacc += v;
      }
      __syncthreads();
    }
    // next super tile's partial sums: loads in flight while this one computes
    if (a.rg_fast && it + 1 < n_iter && wave0 < total)
      rg_issue(a, chain, row0 + rows, row_end, rows, nx, t, e0);
    // ---- this wave's row tile rw of the super tile
    const float* xw = xs + rw * TR * a.xst;
    const float* dw = dfs + rw * TR * a.auxst;
    float xf[8];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) xf[ks] = (ks < KS && 4 * ks < d) ? xw[lr * a.xst + 4 * ks + lq] : 0.f;
    float dff[KGM];
#pragma unroll
    for (int ks = 0; ks < KGM; ++ks) {
      const int o = 4 * ks + lq;
      dff[ks] = (o < g) ? dw[lr * a.auxst + o] : 0.f;
    }
    float dfg[NOT][4];
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = ot * 16 + lr;
        dfg[ot][r] = (o < g) ? dw[(4 * lq + r) * a.auxst + o] : 0.f;
      }
    const int KG = (g + 3) >> 2;
    const float dg1 = G1 ? dw[lr * a.auxst] : 0.f;
    float dg4[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) dg4[r] = G1 ? dw[(4 * lq + r) * a.auxst] : 0.f;
    const int rrow0 = row0 + rw * TR;  // this wave's first row
    const bool live = rrow0 < row_end;  // the group's last super tile may be partly empty
    f4 dxa[4] = {f4zero(), f4zero(), f4zero(), f4zero()};
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      if (!live || !chunk_ok(i)) continue;  // wave-uniform
      const int ci = i * ncw + cw, f0 = chunk_f0(i);
      const float* wsc = wsa + ci * 16 * g;
      const int whalf = nf * g;
      const float* osc = osa + ci * 16;
      float wd0[KGM], wd1[KGM];
      f4 oxv[4];
      if (dphi) {
        const bool frow = f0 + lr < R;
#pragma unroll
        for (int ks = 0; ks < KGM; ++ks) {
          const int o = 4 * ks + lq, wo = lr * g + o;
          const bool ok = o < g && frow;
          wd0[ks] = G1 ? 0.f : (ok ? wsc[wo] : 0.f);
          wd1[ks] = (G1 || !RBF) ? 0.f : (ok ? wsc[whalf + wo] : 0.f);
        }
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
          oxv[dt] = dt < ND ? *reinterpret_cast<const f4*>(osc + (dt * 16 + lr) * a.osa_st + 4 * lq)
                            : f4zero();
      }
      const float* a0 = a0b ? a0b + (int64_t)rrow0 * R + f0 : nullptr;
      f4 at_t;
      if (KS == 0 && a0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) at_t[r] = a0_sum1(a0 + (int64_t)(4 * lq + r) * R + lr, a.a0_sl);
      } else {
        at_t = a_tile<KS, true>(om, R, d, f0, omk[i], xf, xw, a.xst, lr, lq);
      }
      f4 at_n = f4zero(), dpc = f4zero(), dps = f4zero();
      if (dphi) {
        at_n = (KS == 0 && a0) ? a0_sum4(a0 + (int64_t)lr * R + 4 * lq, a.a0_sl)
                               : a_tile<KS, false>(om, R, d, f0, omk[i], xf, xw, a.xst, lr, lq);
        if (G1) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int fl = ci * 16 + 4 * lq + r;
            const bool ok = f0 + 4 * lq + r < R;
            dpc[r] = ok ? dg1 * wsa[fl] : 0.f;
            dps[r] = (ok && RBF) ? dg1 * wsa[whalf + fl] : 0.f;
          }
        } else {
#pragma unroll
          for (int ks = 0; ks < KGM; ++ks) {
            if (ks < KG) {
              dpc = mfma16(wd0[ks], dff[ks], dpc);
              if (RBF) dps = mfma16(wd1[ks], dff[ks], dps);
            }
          }
        }
      }
      float q0[4], q1[4];
      features<RBF>(at_t, cl, q0, q1);
      float da[4];
      if (dphi) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (RBF) {
            float sv, cv;
            rf_sincos(at_n[r], &sv, &cv);
            da[r] = -(cl * sv) * dpc[r] + (cl * cv) * dps[r];
            if (FB) ampl += dpc[r] * (cl * cv) + dps[r] * (cl * sv);
          } else {
            da[r] = at_n[r] > 0.f ? cl * dpc[r] : 0.f;
            if (FB) ampl += dpc[r] * (cl * fmaxf(at_n[r], 0.f));
          }
        }
      }
      // gW_l of this row tile, accumulated over the group
      if (G1) {
        float gc = 0.f, gs = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          gc = fmaf(q0[r], dg4[r], gc);
          if (RBF) gs = fmaf(q1[r], dg4[r], gs);
        }
        gc += __shfl_xor(gc, 16);
        gc += __shfl_xor(gc, 32);
        if (RBF) {
          gs += __shfl_xor(gs, 16);
          gs += __shfl_xor(gs, 32);
        }
        g1c[i] += gc;
        g1s[i] += gs;
      } else {
#pragma unroll
        for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            gacc[i][ot][0] = mfma16(q0[r], dfg[ot][r], gacc[i][ot][0]);
            if (RBF) gacc[i][ot][1] = mfma16(q1[r], dfg[ot][r], gacc[i][ot][1]);
          }
      }
      if (dxw > 0) {
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
          if (dt < ND) {
#pragma unroll
            for (int r = 0; r < 4; ++r) dxa[dt] = mfma16(oxv[dt][r], da[r], dxa[dt]);
          }
      }
      if (FB) {
        float rs = (da[0] + da[1]) + (da[2] + da[3]);
        rs += __shfl_xor(rs, 16);
        rs += __shfl_xor(rs, 32);
        for (int dt = 0; dt * 16 < d; ++dt) {
          f4 zf;
          if (NZ > 0) {
            zf = zpf[i][0];
#pragma unroll
            for (int q = 1; q < NZ; ++q)
              if (dt == q) zf = zpf[i][q];
          } else {
            zf = z_frag(f0, dt);
          }
          f4 dz = f4zero();
#pragma unroll
          for (int r = 0; r < 4; ++r) dz = mfma16(zf[r], da[r], dz);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int kk = dt * 16 + 4 * lq + r;
            const float xv = kk < d ? xw[lr * a.xst + kk] : 0.f;
            const float s1 = sum16(xv * dz[r]);
            const float s2 = sum16(xv * rs);
            if (lr == 0 && kk < d) {
              hw[kk] += s1;
              hw[d + kk] += s2;
            }
          }
        }
      }
    }
    if (it == 0) RG_STAMP(stamp_base, 3);
    // ---- dX of the super tile: the chunk-waves' tiles summed in LDS, stored as the slice partial
    if (dxw > 0) {
      float* redw = red + wave * TR * DP;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        if (dt < ND)
#pragma unroll
          for (int r = 0; r < 4; ++r) redw[lr * DP + dt * 16 + 4 * lq + r] = dxa[dt][r];
      __syncthreads();
      for (int e = threadIdx.x; e < rows * dxw; e += blockDim.x) {
        const int r = e / dxw, k = e - r * dxw, b = row0 + r;
        const int rwi = r >> 4, rr = r & 15;
        if (b < row_end) {
          const float* rp = red + (rwi * ncw) * TR * DP + rr * DP + k;
          float v = rp[0];
          for (int c = 1; c < ncw; ++c) v += rp[c * TR * DP];
          dxp[(int64_t)b * dxw + k] = v;
        }
      }
    }
    __syncthreads();  // LDS tiles free for the next super tile
    if (it == 0) RG_STAMP(stamp_base, 4);
    if (it == 1) RG_STAMP(stamp_base, 5);
  }
  RG_STAMP(stamp_base, 6);

  // ---- the group's gW partial row: row-waves summed in order (LDS), then stored
  float* gwp = a.gwp + (int64_t)chain * a.ws_cs + (int64_t)rg * a.gw_ld;
  constexpr int GSZ = G1 ? NIT * 2 * 64 : NIT * NOT * 2 * 256;  // floats per wave
  float* gred = smem + a.gred_off;
  if (nrw > 1) {
    float* gw = gred + wave * GSZ;
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      if (G1) {
        gw[(i * 2) * 64 + lane] = g1c[i];
        gw[(i * 2 + 1) * 64 + lane] = g1s[i];
      } else {
#pragma unroll
        for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
          for (int h = 0; h < 2; ++h)
            *reinterpret_cast<f4*>(gw + ((i * NOT + ot) * 2 + h) * 256 + 4 * lane) = gacc[i][ot][h];
      }
    }
    __syncthreads();
    if (rw == 0) {
#pragma unroll
      for (int i = 0; i < NIT; ++i) {
        for (int w = 1; w < nrw; ++w) {
          const float* gq = gred + (w * ncw + cw) * GSZ;
          if (G1) {
            g1c[i] += gq[(i * 2) * 64 + lane];
            g1s[i] += gq[(i * 2 + 1) * 64 + lane];
          } else {
#pragma unroll
            for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
              for (int h = 0; h < 2; ++h)
                gacc[i][ot][h] += *reinterpret_cast<const f4*>(gq + ((i * NOT + ot) * 2 + h) * 256 + 4 * lane);
          }
        }
      }
    }
  }
  if (rw == 0) {
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      if (!chunk_ok(i)) continue;
      const int f0 = chunk_f0(i);
      if (G1) {
        const int f = f0 + lr;
        if (lq == 0 && f < R) {
          gwp[f] = g1c[i];
          if (RBF) gwp[R + f] = g1s[i];
        }
      } else {
#pragma unroll
        for (int ot = 0; ot < NOT; ++ot) {
          const int o = ot * 16 + lr;
          if (o < g) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int f = f0 + 4 * lq + r;
              if (f < R) {
                gwp[(int64_t)f * g + o] = gacc[i][ot][0][r];
                if (RBF) gwp[(int64_t)(R + f) * g + o] = gacc[i][ot][1][r];
              }
            }
          }
        }
      }
    }
  }
  RG_STAMP(stamp_base, 7);
  if (FB) {
    // log_amp term over the wave, then the workgroup's partial row [2d+1] in wave order
    float v = sum16(ampl);
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    if (lane == 0) hw[2 * d] = v;
    __syncthreads();
    float* hp = a.hp + (int64_t)chain * a.ws_cs + ((int64_t)rg * NSM + sl) * hst;
    const float* h0 = smem + a.hred_off;
    for (int e = threadIdx.x; e < 2 * d + 1; e += blockDim.x) {
      float s = h0[e];
      for (int w = 1; w < RG_WAVES; ++w) s += h0[w * hst + e];
      hp[e] = s;
    }
    if (a.last && a.lik_fb && threadIdx.x == 0 && sl == 0)
      a.hpl[(int64_t)chain * a.ws_cs + rg] = lvacc;
  }
#ifdef DGPRF_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  RG_STAMP(stamp_base, 14);
}

// launch dispatch: NOT x G1 x RBF x FB x NIT for one KS
template <int KS, int NOT, bool G1>
void k_step_bwd_rg_launch3(bool rbf, bool fb, int nit, dim3 grid, size_t lds, hipStream_t s,
                           const LayerK& a) {
#define DGPRF_BWDRG(R_, F_, I_)                                                                   \
  do {                                                                                           \
    dgprf::set_lds_limit((const void*)k_step_bwd_rg<KS, NOT, R_, G1, F_, I_>, lds);             \
    hipLaunchKernelGGL((k_step_bwd_rg<KS, NOT, R_, G1, F_, I_>), grid, dim3(64 * RG_WAVES), lds, \
                       s, a);                                                                    \
  } while (0)
  if (nit <= 1) {
    if (rbf) {
      if (fb) DGPRF_BWDRG(true, true, 1);
      else DGPRF_BWDRG(true, false, 1);
    } else {
      if (fb) DGPRF_BWDRG(false, true, 1);
      else DGPRF_BWDRG(false, false, 1);
    }
  } else {
    if (rbf) {
      if (fb) DGPRF_BWDRG(true, true, 2);
      else DGPRF_BWDRG(true, false, 2);
    } else {
      if (fb) DGPRF_BWDRG(false, true, 2);
      else DGPRF_BWDRG(false, false, 2);
    }
  }
#undef DGPRF_BWDRG
}
template <int KS>
void k_step_bwd_rg_launch2(int g, bool rbf, bool fb, int nit, dim3 grid, size_t lds, hipStream_t s,
                           const LayerK& a) {
  const int NOT = (g + 15) >> 4;
  if (g == 1) k_step_bwd_rg_launch3<KS, 1, true>(rbf, fb, nit, grid, lds, s, a);
  else if (NOT == 1) k_step_bwd_rg_launch3<KS, 1, false>(rbf, fb, nit, grid, lds, s, a);
  else if (NOT == 2) k_step_bwd_rg_launch3<KS, 2, false>(rbf, fb, nit, grid, lds, s, a);
  else if (NOT == 3) k_step_bwd_rg_launch3<KS, 3, false>(rbf, fb, nit, grid, lds, s, a);
  else k_step_bwd_rg_launch3<KS, 4, false>(rbf, fb, nit, grid, lds, s, a);
}

}  // namespace dgprf_sk

#ifdef DGPRF_KS
template void dgprf_sk::k_step_bwd_rg_launch2<DGPRF_KS>(int, bool, bool, int, dim3, size_t,
                                                        hipStream_t, const dgprf_sk::LayerK&);
#endif
