// step_bwdrw_impl.h — the row-wave step backward k_step_bwd_rw, included by step_bwdrw_k<KS>.hip.
//
// The row-group backward (step_bwdrg_impl.h) for narrow slices (at most 8 accumulator tiles of gW
// per slice: config 2's RBF n_rf 1024 / g 8, config 3's ARC n_rf 2048 / g 9) after the fused
// all-layer forward (complete F_l, plan rt_per_group >= 8): every wave of an 8-wave workgroup owns
// the WHOLE feature slice for its own row tiles (rt0 + w, rt0 + w + 8, ...), so
//   * a wave's dX rows are complete slice sums in its own registers — stored straight to the slice
//     partial, no cross-wave LDS reduction;
//   * its X / dF tiles live in a wave-private LDS region (the next tile's partial sums prefetched
//     into registers while the current one computes);
//   * nothing in the row-tile loop waits for another wave: no workgroup barrier until the end,
//     where the 8 waves' gW accumulators are summed in LDS in wave order and the group's gW
//     partial row is written (one row per group, <= 16 whatever B, as in the row-group kernel).
// Same arithmetic as k_step_bwd (analytic tape.gradient, models/dgp.py:194-198).  Deterministic:
// fixed row-tile order inside each wave's accumulators, then waves 0..7.
#pragma once
#include "step_common.h"

namespace dgprf_sk {

constexpr int RW_TS = 20;  // row stride of a wave's 16 x 16 transpose scratch (16-byte rows)

// -DDGPRF_STAMPS diagnostic build only: s_memtime of lane 0 of a chosen wave into a.stamps
#ifdef DGPRF_STAMPS
#define RW_STAMP(cond, i)                                                               \
  do {                                                                                 \
    if ((cond) && (threadIdx.x & 63) == 0 && a.stamps) {                               \
      __builtin_amdgcn_sched_barrier(0);                                               \
      a.stamps[(size_t)stamp_base * 16 + (i)] = __builtin_amdgcn_s_memtime();          \
      __builtin_amdgcn_sched_barrier(0);                                               \
    }                                                                                  \
  } while (0)
#else
#define RW_STAMP(cond, i) \
  do {                    \
  } while (0)
#endif

// NCH: 16-feature chunks of the slice (4 cpw); EX / ED: prefetched X / dF elements per lane
// (16 dpad / 64, 16 g / 64 rounded up).
// DX: the layer has a dX output (l > 0; dxw <= 16, one 16-wide dX tile).  Compile-time so the
// chunk body carries no runtime branch: KG = ED dF k-steps, slices of whole chunks (R % nf == 0).
template <int KS, int NOT, bool RBF, bool G1, bool FB, int NCH, int ED, int NWV, bool DX>
__global__ __launch_bounds__(64 * NWV) void k_step_bwd_rw(const LayerK a) {
  constexpr int EX = KS;  // 16 rows x 4 KS columns of X = KS elements per lane
  extern __shared__ __attribute__((aligned(16))) float smem[];
  int rg, sl;
  if (!tile_of_block(a, rg, sl)) return;
  const int chain = blockIdx.z;
#ifdef DGPRF_STAMPS
  const int stamp_base = (a.layer * 2 + 1) * 4096 + blockIdx.z * gridDim.x + blockIdx.x;
#endif
  const float* __restrict__ om = a.om + (int64_t)chain * a.om_cs;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, lr = lane & 15, lq = lane >> 4;
  const int R = a.R, g = a.g, d = a.d, B = a.B, dxw = a.dxw;
  const int nf = 64 * a.cpw, fb0 = sl * nf;
  const int n_rt_all = (B + TR - 1) / TR;
  const int rt0 = rg * a.rt_per_rg;
  const int rt_end = min(rt0 + a.rt_per_rg, n_rt_all);
  const int row_end = min(rt_end * TR, B);
  constexpr int KGM = 4 * NOT;
  constexpr int KG = ED;  // dF k-steps: ceil(g / 4) (rw_config: ED = ceil(16 g / 64))
  constexpr bool dphi = FB || DX;
  constexpr int GPW = G1 ? 1 : 4 * KG;  // W staging row width (outputs, zero past g)
  const int xst = a.xst, dst = a.auxst;  // 4 KS + 1, 17 (rw_config)
  float* wsa = smem + a.wsa_off;               // [RBF ? 2 : 1][nf][GPW]
  float* osa = smem + a.osa_off;               // [max(4 KS, d)][osa_st], zero rows past d
  float* xw = smem + a.aux_off + wave * a.red_off;  // wave-private: X [16][xst], dF, Y [16][dst]
  float* dw = xw + round4(TR * xst);
  float* yw = dw + round4(TR * dst);
  float* tw = yw + round4(TR * dst);            // dA tile transpose scratch [16][RW_TS]
  const float cl = a.cptr[(int64_t)chain * a.der_cs];
  RW_STAMP(wave == 0, 0);

  // ---- the slice's W rows (both halves, outputs zero-padded to GPW) and Omega rows (zero past
  // d), once; the slice holds whole chunks (R % nf == 0)
  {
    const float* W = a.W + (int64_t)chain * a.w_cs;
    constexpr int NH = RBF ? 2 : 1;
    if (dphi)
      for (int e = threadIdx.x; e < NH * nf * GPW; e += blockDim.x) {
        const int h = e / (nf * GPW), r2 = e - h * nf * GPW, f = r2 / GPW, o = r2 - f * GPW;
        wsa[e] = o < g ? W[((int64_t)h * R + fb0 + f) * g + o] : 0.f;
      }
    const int orows = a.rw_orows > dxw ? a.rw_orows : dxw;
    for (int e = threadIdx.x; e < orows * nf; e += blockDim.x) {
      const int k = e / nf, c = e - k * nf;
      osa[k * a.osa_st + c] = k < d ? om[(int64_t)k * R + fb0 + c] : 0.f;
    }
  }
  // the wave's tiles: zero once, so the X columns >= d and dF / Y columns >= g read as zeros
  for (int e = lane; e < round4(TR * xst) + 2 * round4(TR * dst); e += 64) xw[e] = 0.f;
  constexpr int NZ = (4 * KS + 15) / 16;
  const rsrc_t rz = make_rsrc(a.z, FB ? (int64_t)d * R : 0);
  f4 zpf[NCH][FB ? NZ : 1];
  if (FB)
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int dt = 0; dt < NZ; ++dt) {
        const int k = dt * 16 + lr, f0 = fb0 + c * 16;
        zpf[c][dt] = bload4(rz, k < d && f0 + 4 * lq < R ? (uint32_t)(((int64_t)k * R + f0 + 4 * lq) * 4)
                                                          : DGPRF_OOB);
      }

  f4 gacc[NCH][NOT][2];
  float g1c[NCH], g1s[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    g1c[c] = g1s[c] = 0.f;
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot) gacc[c][ot][0] = gacc[c][ot][1] = f4zero();
  }
  const int hst = round4(2 * d + 1);
  float* hw = smem + a.hred_off + wave * hst;
  float ampl = 0.f, lvacc = 0.f;
  if (FB)
    for (int e = lane; e < hst; e += 64) hw[e] = 0.f;

  // ---- prefetch of one row tile: X (complete F_{l-1} | dataset columns; KS x 4 columns, lane
  // owns column 4 ks + lq of row lr) and dF (16 slices of dX_{l+1}, or complete F_L; element
  // u = lane + 64 e of the [16][g] tile)
  const rsrc_t rws = make_rsrc(a.ws + (int64_t)chain * a.ws_cs, a.ws_cs);
  const rsrc_t rxd = make_rsrc(a.xrows + (int64_t)chain * a.xrow_cs, (int64_t)B * (d - a.gp));
  const rsrc_t ry = make_rsrc(a.yrows + (int64_t)chain * a.yrow_cs, (int64_t)B * a.y_cols);
  // F_L complete (fused forward) / dX_{l+1} slice partials.  Written as a.last || a.rw_one (the
  // host sets rw_one = last): from a.last alone the compiler versions the prefetch per case (68
  // instead of 54 buffer loads, 127 instead of 108 branches) and the B = 65,536 step's layer-0
  // backward took 127 instead of 93 us; from a count argument it spills 55 instead of 21 SGPRs
  const int nsl = (a.last || a.rw_one) ? 1 : NSM;
  const int yc = a.likelihood == DGPRF_LIK_GAUSSIAN ? g : 1;
  float px[EX], pd[ED][NSM], py[ED];
  auto issue = [&](int rt) {
    const int row0 = rt * TR;
#pragma unroll
    for (int e = 0; e < EX; ++e) {
      const int k = 4 * e + lq, b = row0 + lr;
      const bool ok = b < row_end && k < d;
      // both sources loaded (one OOB-masked to 0) and added: a per-lane choice between the two
      // descriptors would compile to a waterfall loop around the load
      const float vf = bload1(rws, ok && k < a.gp ? (uint32_t)((a.fprev_off + b * a.gp + k) * 4) : DGPRF_OOB);
      const float vd = bload1(rxd, ok && k >= a.gp ? (uint32_t)((b * (d - a.gp) + (k - a.gp)) * 4) : DGPRF_OOB);
      px[e] = vf + vd;
    }
#pragma unroll
    for (int e = 0; e < ED; ++e) {
      const int u = lane + 64 * e, r = u / g, o = u - r * g, b = row0 + r;
      const bool ok = u < TR * g && b < row_end;
#pragma unroll
      for (int s = 0; s < NSM; ++s)
        pd[e][s] = bload1(rws, ok && s < nsl ? (uint32_t)((a.dsrc_off + s * B * g + b * g + o) * 4)
                                              : DGPRF_OOB);
      py[e] = bload1(ry, ok && a.last ? (uint32_t)((b * a.y_cols + min(o, yc - 1)) * 4) : DGPRF_OOB);
    }
  };
  const int dpad = round4(d);  // the X tile row holds columns < dpad (xst = dpad + 1)
  auto commit = [&]() {
#pragma unroll
    for (int e = 0; e < EX; ++e)
      if (4 * e + lq < dpad) xw[lr * xst + 4 * e + lq] = px[e];
#pragma unroll
    for (int e = 0; e < ED; ++e) {
      const int u = lane + 64 * e, r = u / g, o = u - r * g;
      float v = pd[e][0];
#pragma unroll
      for (int s = 1; s < NSM; ++s) v += pd[e][s];
      if (u < TR * g) {
        dw[r * dst + o] = v;
        yw[r * dst + o] = py[e];
      }
    }
  };

  float* dxp = a.dxout + (int64_t)chain * a.ws_cs + (int64_t)sl * B * dxw;
  __syncthreads();  // staged slice visible to every wave
  RW_STAMP(wave == 0, 1);
  int rt = rt0 + wave;
  // 8 waves: the next row tile's loads are prefetched into registers while this one computes;
  // 16 waves (four per SIMD, 128 VGPRs): no prefetch registers, the other waves hide the loads
  constexpr bool PF = NWV == 8;
  if (PF && rt < rt_end) issue(rt);
  int it = 0;
  for (; rt < rt_end; rt += NWV, ++it) {
    const int row0 = rt * TR;
    RW_STAMP(wave == 0 && it < 3, 2 + 3 * it);
    if (!PF) issue(rt);
    commit();
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes done
    __builtin_amdgcn_wave_barrier();
    RW_STAMP(wave == 0 && it < 3, 3 + 3 * it);
    if (a.last) {
      // likelihood gradient dF = -(1/B) dlogp/dF (likelihoods/gaussian.py:18-25, softmax.py:8-15)
      float lvrow = 0.f;
      if (lane < TR) {
        const int b = row0 + lane;
        float* df = dw + lane * dst;
        if (b < row_end) {
          const float* y = yw + lane * dst;
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
      if (FB && a.lik_fb) lvacc += sum16(lvrow);
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
    }
    // the next row tile's loads are in flight while this one computes
    if (PF && rt + NWV < rt_end) issue(rt + NWV);
    float xf[8];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) xf[ks] = ks < KS ? xw[lr * xst + 4 * ks + lq] : 0.f;
    float dff[KGM];
#pragma unroll
    for (int ks = 0; ks < KG; ++ks) dff[ks] = dw[lr * dst + 4 * ks + lq];  // zero past g
    float dfg[NOT][4];
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
      for (int r = 0; r < 4; ++r) dfg[ot][r] = dw[(4 * lq + r) * dst + ot * 16 + lr];
    float dg4[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) dg4[r] = G1 ? dw[(4 * lq + r) * dst] : 0.f;
    f4 dxa = f4zero();
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int f0 = fb0 + c * 16;  // < R: slices hold whole chunks (rw_config)
      const float* wsc = wsa + c * 16 * GPW;
      const int whalf = nf * GPW;
      const float* osc = osa + c * 16;
      // Omega fragments of the A tile from the staged rows: omk[ks] = Omega[4 ks + lq][f0 + lr]
      float omk[8];
#pragma unroll
      for (int ks = 0; ks < 8; ++ks)
        omk[ks] = ks < KS ? osc[(4 * ks + lq) * a.osa_st + lr] : 0.f;  // zero rows past d
      float wd0[KGM], wd1[KGM];
      f4 oxv = f4zero();
      if (dphi) {
#pragma unroll
        for (int ks = 0; ks < KG; ++ks) {
          const int wo = lr * GPW + 4 * ks + lq;
          wd0[ks] = G1 ? 0.f : wsc[wo];
          wd1[ks] = (G1 || !RBF) ? 0.f : wsc[whalf + wo];
        }
      }
      if (DX) oxv = *reinterpret_cast<const f4*>(osc + lr * a.osa_st + 4 * lq);
      // A tile in the rows-in-registers orientation: at_t[r] = A[row 4 lq + r][f0 + lr]
      const f4 at_t = a_tile<KS, true>(om, R, d, f0, omk, xf, xw, xst, lr, lq);
      // dPhi in the same orientation: dpc[r] = dPhi_cos[row 4 lq + r][f0 + lr] = sum_o dF W
      f4 dpc = f4zero(), dps = f4zero();
      if (dphi) {
        if (G1) {
          const float w0 = wsc[lr], w1 = RBF ? wsc[whalf + lr] : 0.f;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            dpc[r] = dg4[r] * w0;
            dps[r] = dg4[r] * w1;
          }
        } else {
#pragma unroll
          for (int ks = 0; ks < KG; ++ks) {
            dpc = mfma16(dff[ks], wd0[ks], dpc);
            if (RBF) dps = mfma16(dff[ks], wd1[ks], dps);
          }
        }
      }
      float q0[4], q1[4];
      features<RBF>(at_t, cl, q0, q1);  // q0 = c cos A | c relu A, q1 = c sin A
      float da[4];
      if (dphi) {
        float dat[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (RBF) {
            dat[r] = -q1[r] * dpc[r] + q0[r] * dps[r];
            if (FB) ampl += dpc[r] * q0[r] + dps[r] * q1[r];
          } else {
            dat[r] = at_t[r] > 0.f ? cl * dpc[r] : 0.f;
            if (FB) ampl += dpc[r] * q0[r];
          }
        }
        // dA to the features-in-registers orientation of the dX / z contractions through the
        // wave's LDS scratch: da[r] = dA[row lr][f0 + 4 lq + r]
        *reinterpret_cast<f4*>(tw + lr * RW_TS + 4 * lq) = f4{dat[0], dat[1], dat[2], dat[3]};
#pragma unroll
        for (int r = 0; r < 4; ++r) da[r] = tw[(4 * lq + r) * RW_TS + lr];
      }
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
        g1c[c] += gc;
        g1s[c] += gs;
      } else {
#pragma unroll
        for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            gacc[c][ot][0] = mfma16(q0[r], dfg[ot][r], gacc[c][ot][0]);
            if (RBF) gacc[c][ot][1] = mfma16(q1[r], dfg[ot][r], gacc[c][ot][1]);
          }
      }
      if (DX) {
#pragma unroll
        for (int r = 0; r < 4; ++r) dxa = mfma16(oxv[r], da[r], dxa);
      }
      if (FB) {
        float rs = (da[0] + da[1]) + (da[2] + da[3]);
        rs += __shfl_xor(rs, 16);
        rs += __shfl_xor(rs, 32);
#pragma unroll
        for (int dt = 0; dt < NZ; ++dt) {
          f4 dz = f4zero();
#pragma unroll
          for (int r = 0; r < 4; ++r) dz = mfma16(zpf[c][dt][r], da[r], dz);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int kk = dt * 16 + 4 * lq + r;
            const float xv = kk < d ? xw[lr * xst + kk] : 0.f;
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
    RW_STAMP(wave == 0 && it < 3, 4 + 3 * it);
    // dX rows of this tile: the slice's complete sum (dxa[r] = dX[row lr][4 lq + r])
    if (DX) {
      const int b = row0 + lr;
      if (b < row_end) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int k = 4 * lq + r;
          if (k < dxw) dxp[(int64_t)b * dxw + k] = dxa[r];
        }
      }
    }
  }

  RW_STAMP(wave == NWV - 1, 13);
  RW_STAMP(wave == 0, 11);
  // ---- the group's gW partial row: the waves' accumulators summed in a fixed order — 8 LDS
  // slots, slot w = wave w (+ wave w + 8 with 16 waves), then slots 0..7
  __syncthreads();
  RW_STAMP(wave == 0, 12);
  constexpr int HN = RBF ? 2 : 1;  // cos | sin halves (RBF), one half (ARC)
  constexpr int GSZ = G1 ? NCH * 2 * 64 : NCH * NOT * HN * 256;
  constexpr int NSLOT = 8;
  float* gred = smem + a.gred_off;
  auto put = [&](bool add) {
    float* gw = gred + (wave & (NSLOT - 1)) * GSZ;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      if (G1) {
        float* p0 = gw + (c * 2) * 64 + lane;
        float* p1 = gw + (c * 2 + 1) * 64 + lane;
        *p0 = add ? *p0 + g1c[c] : g1c[c];
        *p1 = add ? *p1 + g1s[c] : g1s[c];
      } else {
#pragma unroll
        for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
          for (int h = 0; h < HN; ++h) {
            f4* p = reinterpret_cast<f4*>(gw + ((c * NOT + ot) * HN + h) * 256 + 4 * lane);
            *p = add ? *p + gacc[c][ot][h] : gacc[c][ot][h];
          }
      }
    }
  };
  if (wave < NSLOT) put(false);
  if (FB) {
    float v = sum16(ampl);
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    if (lane == 0) {
      hw[2 * d] = v;
      hw[2 * d + 1] = lvacc;  // padding slot of the wave's row (hst >= 2 d + 2)
    }
  }
  __syncthreads();
  if (NWV > NSLOT) {
    if (wave >= NSLOT) put(true);
    __syncthreads();
  }
  // every thread sums a strided share of the gW values in slot order and stores them
  float* gwp = a.gwp + (int64_t)chain * a.ws_cs + (int64_t)rg * a.gw_ld;
  if (G1) {
    for (int e = threadIdx.x; e < NCH * 2 * 16; e += blockDim.x) {
      const int c = e / 32, h = (e / 16) & 1, fl = e & 15;  // lanes 0..15 hold features fl
      float v = gred[(c * 2 + h) * 64 + fl];
      for (int w = 1; w < NSLOT; ++w) v += gred[w * GSZ + (c * 2 + h) * 64 + fl];
      const int f = fb0 + c * 16 + fl;
      if (f < R && (h == 0 || RBF)) gwp[h * R + f] = v;
    }
  } else {
    for (int e = threadIdx.x; e < GSZ; e += blockDim.x) {
      // e = ((c NOT + ot) HN + h) 256 + 4 lane + r: gacc[c][ot][h][r] of lane
      const int blk = e >> 8, within = e & 255, ln = within >> 2, r = within & 3;
      const int h = blk % HN, ot = (blk / HN) % NOT, c = (blk / HN) / NOT;
      float v = gred[e];
      for (int w = 1; w < NSLOT; ++w) v += gred[w * GSZ + e];
      // gacc[c][ot][h][r] of lane ln = gW[f0 + 4 (ln >> 4) + r][ot 16 + (ln & 15)] (half h)
      const int f = fb0 + c * 16 + 4 * (ln >> 4) + r, o = ot * 16 + (ln & 15);
      if (f < R && o < g) gwp[(int64_t)(h * R + f) * g + o] = v;
    }
  }
  if (FB) {
    float* hp = a.hp + (int64_t)chain * a.ws_cs + ((int64_t)rg * NSM + sl) * hst;
    const float* h0 = smem + a.hred_off;
    for (int e = threadIdx.x; e < 2 * d + 1; e += blockDim.x) {
      float s = h0[e];
      for (int w = 1; w < NWV; ++w) s += h0[w * hst + e];
      hp[e] = s;
    }
    if (a.last && a.lik_fb && threadIdx.x == 0 && sl == 0) {
      float s = h0[2 * d + 1];
      for (int w = 1; w < NWV; ++w) s += h0[w * hst + 2 * d + 1];
      a.hpl[(int64_t)chain * a.ws_cs + rg] = s;
    }
  }
  RW_STAMP(wave == 0, 14);
}

template <int KS, int NOT, bool G1, int NCH, int ED, int NWV, bool RBF>
void k_step_bwd_rw_launch4(bool fb, bool dx, dim3 grid, size_t lds, hipStream_t s, const LayerK& a) {
#define DGPRF_BWDRW(F_, D_)                                                                         \
  do {                                                                                             \
    dgprf::set_lds_limit((const void*)k_step_bwd_rw<KS, NOT, RBF, G1, F_, NCH, ED, NWV, D_>, lds);  \
    hipLaunchKernelGGL((k_step_bwd_rw<KS, NOT, RBF, G1, F_, NCH, ED, NWV, D_>), grid,               \
                       dim3(64 * NWV), lds, s, a);                                                 \
  } while (0)
  if (fb) {
    if (dx) DGPRF_BWDRW(true, true);
    else DGPRF_BWDRW(true, false);
  } else {
    if (dx) DGPRF_BWDRW(false, true);
    else DGPRF_BWDRW(false, false);
  }
#undef DGPRF_BWDRW
}
template <int KS, int NWV>
void k_step_bwd_rw_launch3(int g, bool rbf, bool fb, bool dx, int nch, dim3 grid, size_t lds,
                           hipStream_t s, const LayerK& a) {
  const int ed = (16 * g + 63) / 64;
  // RBF slices hold 4 chunks (8 accumulator tiles: cos | sin), ARC slices 4 or 8
#define DGPRF_RW_ED(G1_, NCH_, R_)                                                                 \
  do {                                                                                            \
    if (G1_) k_step_bwd_rw_launch4<KS, 1, true, NCH_, 1, NWV, R_>(fb, dx, grid, lds, s, a);        \
    else if (ed <= 1) k_step_bwd_rw_launch4<KS, 1, false, NCH_, 1, NWV, R_>(fb, dx, grid, lds, s, a); \
    else if (ed == 2) k_step_bwd_rw_launch4<KS, 1, false, NCH_, 2, NWV, R_>(fb, dx, grid, lds, s, a); \
    else k_step_bwd_rw_launch4<KS, 1, false, NCH_, 3, NWV, R_>(fb, dx, grid, lds, s, a);          \
  } while (0)
  if (rbf) {
    if (g == 1) DGPRF_RW_ED(true, 4, true);
    else DGPRF_RW_ED(false, 4, true);
  } else if (nch == 4) {
    if (g == 1) DGPRF_RW_ED(true, 4, false);
    else DGPRF_RW_ED(false, 4, false);
  } else {
    if (g == 1) DGPRF_RW_ED(true, 8, false);
    else DGPRF_RW_ED(false, 8, false);
  }
#undef DGPRF_RW_ED
}
// g <= 12 (ED = ceil(16 g / 64) <= 3), 4 or 8 chunks per slice, 8 or 16 waves
template <int KS>
void k_step_bwd_rw_launch2(int g, bool rbf, bool fb, bool dx, int nch, int nwv, dim3 grid,
                           size_t lds, hipStream_t s, const LayerK& a) {
  if (nwv == 16) k_step_bwd_rw_launch3<KS, 16>(g, rbf, fb, dx, nch, grid, lds, s, a);
  else k_step_bwd_rw_launch3<KS, 8>(g, rbf, fb, dx, nch, grid, lds, s, a);
}

}  // namespace dgprf_sk

#ifdef DGPRF_KS
template void dgprf_sk::k_step_bwd_rw_launch2<DGPRF_KS>(int, bool, bool, bool, int, int, dim3,
                                                        size_t, hipStream_t, const dgprf_sk::LayerK&);
#endif
