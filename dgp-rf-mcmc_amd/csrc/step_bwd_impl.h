// step_bwd_impl.h — the step backward kernel k_step_bwd (the analytic form of tape.gradient,
// models/dgp.py:194-198, for one layer: likelihood gradient, gW_l = Phi_l^T dF_l, dPhi, dA, dX_l)
// and its launch dispatch, included by step_bwd_k<KS>.hip.
#pragma once
#include "step_common.h"

namespace dgprf_sk {

// Whole-slice staging (a.wstage): W rows [fb0, fb0 + 64 cpw) of both halves (contiguous runs of
// 64 cpw g floats in W) and Omega rows k < dxw over the same features (runs of 64 cpw floats, one
// LDS row of 64 cpw + 4 each) as 16-byte global_load_lds: lane-linear LDS destinations, no VGPRs,
// every copy in flight at once; the prologue's barrier waits for them.  The slice lies inside the
// layer (R % (64 cpw) == 0) and every run starts 16-byte aligned (R g % 4 == 0).
__device__ __forceinline__ void stage_slice_lds(const LayerK& a, const float* W, const float* om,
                                                int fb0, float* smem) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nf = 64 * a.cpw, g = a.g, R = a.R;
  const int n4 = nf * g / 4;  // float4 per half
  const int nh = a.kind_rbf ? 2 : 1;
  for (int h = 0; h < nh; ++h) {
    const float* src = W + ((int64_t)h * R + fb0) * g;
    float* dst = smem + a.wsa_off + h * nf * g;
    for (int i0 = wave * 64; i0 < n4; i0 += (int)blockDim.x) {
      if (i0 + lane < n4)
        __builtin_amdgcn_global_load_lds(src + 4 * (i0 + lane), dst + 4 * i0, 16, 0, 0);
    }
  }
  const int per_row = nf / 256;  // 256-float instructions per Omega row (cpw >= 4)
  for (int j = wave; j < a.dxw * per_row; j += (int)(blockDim.x >> 6)) {
    const int k = j / per_row, c = j - k * per_row;
    __builtin_amdgcn_global_load_lds(om + (int64_t)k * R + fb0 + c * 256 + 4 * lane,
                                     smem + a.osa_off + k * a.osa_st + c * 256, 16, 0, 0);
  }
}


// Folded output layer (a.rcf, RCF instances; step_fold_out): the layer's whole W_L [P] and Omega_L
// rows [d][R + 16] copied global -> LDS with global_load_lds at kernel start (no VGPRs; in flight
// with the prologue's partial-sum loads, waited for by its barrier).  W_L and Omega_L rows start
// 16-byte aligned (w_off / omega_off multiples of 4) and R % 256 == 0.
template <bool RBF>
__device__ __forceinline__ void rcf_stage(const LayerK& a, const float* W, const float* om,
                                          float* smem) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = (int)(blockDim.x >> 6);
  const int R = a.R, P = RBF ? 2 * R : R, per_row = R >> 8;
  float* wl = smem + a.rcf_off;
  float* ol = wl + P;
  for (int j = wave; j < (P >> 8); j += nw)
    __builtin_amdgcn_global_load_lds(W + j * 256 + 4 * lane, wl + j * 256, 16, 0, 0);
  for (int j = wave; j < a.d * per_row; j += nw) {
    const int k = j / per_row, c = j - k * per_row;
    __builtin_amdgcn_global_load_lds(om + (int64_t)k * R + c * 256 + 4 * lane,
                                     ol + k * (R + 16) + c * 256, 16, 0, 0);
  }
}

// This wave's share of F_L[row lr] = sum_f Phi[lr][f] W_L[f] (layers/rf_layers.py:42-44,
// layers/GP_weight_layers.py:11-15, g_L = 1): 16-feature chunks wave, wave + nw, ... in order (nw
// waves in the workgroup), the A tile on v_mfma_f32_16x16x4_f32 from the staged Omega_L rows and the
// X tile, features and the W_L dot product as in k_step_fwd's g = 1 body; summed over the lane's 4
// features then the 4 feature groups (every lane of row lr ends with the same value).
template <int KS, bool RBF>
__device__ __forceinline__ float rcf_row_partial(const LayerK& a, const float* smem,
                                                 const float (&xf)[8], float cl, int wave, int nw,
                                                 int lr, int lq) {
  const int R = a.R, d = a.d, ost = R + 16, nch = R >> 4;
  const float* wl = smem + a.rcf_off;
  const float* ol = wl + (RBF ? 2 * R : R);
  float acc = 0.f;
  // four chunks per group (c0, c0 + nw, c0 + 2 nw, c0 + 3 nw: R % (64 nw) == 0, so every wave's
  // chunk count is a multiple of 4): their A-tile chains are issued together, then the four chunks'
  // features and dot products — independent dependency chains to overlap
  for (int c0 = wave; c0 < nch; c0 += 4 * nw) {
    f4 at[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int f0 = (c0 + nw * q) * 16;
      at[q] = f4zero();
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int k = 4 * ks + lq;
        const float o = ol[(k < d ? k : d - 1) * ost + f0 + lr];  // rows >= d: not staged
        at[q] = mfma16(k < d ? o : 0.f, xf[ks], at[q]);  // at[r] = A[row lr][f0 + 4 lq + r]
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int f0 = (c0 + nw * q) * 16;
      float p0[4], p1[4];
      features<RBF>(at[q], cl, p0, p1);
      const f4 w0 = *reinterpret_cast<const f4*>(wl + f0 + 4 * lq);
      f4 w1 = f4zero();
      if (RBF) w1 = *reinterpret_cast<const f4*>(wl + R + f0 + 4 * lq);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        acc = fmaf(p0[r], w0[r], acc);
        if (RBF) acc = fmaf(p1[r], w1[r], acc);
      }
    }
  }
  acc += __shfl_xor(acc, 16);
  acc += __shfl_xor(acc, 32);
  return acc;
}

// NWB: waves per workgroup (8: W-only, whole-slice LDS image).  GSM: how the gW partial tile
// leaves (1 < g): 0 = chosen at run time (g % 16 == 0: transposed tile, 16-byte lanes; else dword
// stores from the MFMA tile), 1 = transposed tile only, 2 = staged per wave in LDS and stored as
// contiguous 16-byte lanes only (a.gst_off).
// RCF: the folded output layer's instance (g = 1, W-only, NWB = 4): F_L recomputed here, by 4 or
// (R % 512 == 0) 8 waves — waves 4-7 join the copy of the layer, the prologue and the recompute, then
// leave; the rest of the backward is the 4-wave body.
template <int KS, int NOT, bool RBF, bool G1, bool FB, int NWB, int GSM, bool RCF = false>
__global__ __launch_bounds__(RCF ? 512 : 64 * NWB) __attribute__((amdgpu_waves_per_eu((NOT == 1 && !FB && (KS == 1 || KS == 2 || (KS == 4 && !RBF))) ? STEP_WPE : 1))) void k_step_bwd(const LayerK a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr bool WST = NWB == 8;  // whole-slice staging (a.wstage == 1 exactly then)
  int rt, sl;
  if (!tile_of_block(a, rt, sl)) return;
  const int chain = blockIdx.z;
  const float* __restrict__ om = a.om + (int64_t)chain * a.om_cs;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, lr = lane & 15, lq = lane >> 4;
  const int R = a.R, g = a.g, d = a.d, B = a.B, cpw = a.cpw, dxw = a.dxw;
  const int row0 = rt * TR;
  const int stamp_base = (a.layer * 2 + 1) * 4096 + blockIdx.z * gridDim.x + blockIdx.x;
  STEP_STAMP(stamp_base, 0);
  float* xs = smem;
  float* dfs = smem + a.aux_off;
  const int dfst = a.auxst;
  float* red = smem + a.red_off;
  const float* __restrict__ W = a.W + (int64_t)chain * a.w_cs;
  // iteration i of wave w takes chunk i NWB + w of the slice (8-wave workgroups: whole-slice
  // staging only, a.wstage)
  auto chunk_f0 = [&](int i) { return ((sl * cpw * 4 + i * NWB) + wave) * 16; };
  const int nit = cpw * 4 / NWB;
  constexpr int KGM = 4 * NOT;  // k-steps of the dPhi contraction (K = g)
  const int ND = (dxw + 15) >> 4;
  // dX tiles held per lane: dxw = g_{l-1} <= d_l, so at most ceil(4 KS / 16) of them (KS > 0)
  constexpr int NDM = KS == 0 ? 4 : (KS + 3) / 4;
  // dPhi / dA are needed for dX (l > 0) and, with full_bayesian=True, for every layer
  const bool dphi = FB || dxw > 0;

  // first chunk's fragments, issued before the dependent partial sums
  float omk[8];
  if (KS > 0) load_om_frag<KS>(om, R, d, chunk_f0(0), lr, lq, omk);
  // full_bayesian=True: z fragments of the Dz = dA z^T tiles (d <= 32 when KS > 0: two 16-dim
  // tiles prefetched with the Omega fragments; wider layers load them in the chunk loop)
  constexpr int NZ = KS > 0 ? (4 * KS + 15) / 16 : 0;
  const rsrc_t rz = make_rsrc(a.z, FB ? (int64_t)d * R : 0);
  auto z_frag = [&](int f0, int dt) -> f4 {
    const int k = dt * 16 + lr;
    return bload4(rz, k < d && f0 + 4 * lq < R ? (uint32_t)(((int64_t)k * R + f0 + 4 * lq) * 4)
                                               : DGPRF_OOB);
  };
  f4 zpf[NZ > 0 ? NZ : 1];
  if (FB)
#pragma unroll
    for (int dt = 0; dt < NZ; ++dt) zpf[dt] = z_frag(chunk_f0(0), dt);
  // dPhi / dX A operands (W_l rows and Omega_l rows of this workgroup's 64-feature block) are
  // staged through LDS as W [2][64*g] (raw rows) and Omega [rows][OST]; the fragment reads zero
  // feature rows >= R.
  float* wsl = smem + a.stg_off;
  float* osl = smem + a.os_off;
  const int nwh = 64 * g, nwt = RBF ? 2 * nwh : nwh, nom = dxw * 64;
  // general path: clamped scalar loads (contiguous runs), used when a.fast == 0 and for cpw > 1
  constexpr int NJW = 8 * NOT;  // >= 2*64*g/256
  constexpr int NJO = 16;       // >= 64*64/256
  float stw[NJW], sto[NJO];
  auto stage_load = [&](int fb) {
    const int64_t rg = (int64_t)R * g;
#pragma unroll
    for (int j = 0; j < NJW; ++j) {
      const int e = min((int)threadIdx.x + 256 * j, nwt - 1);
      const int h = e >= nwh, e2 = e - h * nwh;
      stw[j] = W[h * rg + min((int64_t)fb * g + e2, rg - 1)];
    }
#pragma unroll
    for (int j = 0; j < NJO; ++j) {
      const int e = min((int)threadIdx.x + 256 * j, max(nom - 1, 0));
      sto[j] = om[(int64_t)(e >> 6) * R + min(fb + (e & 63), R - 1)];
    }
  };
  auto stage_store = [&](int fb) {
#pragma unroll
    for (int j = 0; j < NJW; ++j) {
      const int e = (int)threadIdx.x + 256 * j;
      if (e < nwt) wsl[e] = stw[j];
    }
#pragma unroll
    for (int j = 0; j < NJO; ++j) {
      const int e = (int)threadIdx.x + 256 * j;
      if (e < nom) osl[(e >> 6) * OST + (e & 63)] = fb + (e & 63) < R ? sto[j] : 0.f;
    }
  };
  const int fb0 = (sl * cpw) * 64;
  const float cl = a.cptr[(int64_t)chain * a.der_cs];
  const float* fpl = a.fout + (int64_t)chain * a.ws_cs;        // F_L partials (last layer)
  const float* dxn = a.dxnext + (int64_t)chain * a.ws_cs;      // dX_{l+1} partials
  const float* yr = a.yrows + (int64_t)chain * a.yrow_cs;
  float* ysh = dfs + round4(TR * dfst);
  const int yc = a.likelihood == DGPRF_LIK_GAUSSIAN ? g : 1;
  if (a.fast) {
    // ---- single burst: W/Omega block, X tile, dF (or F_L) partials and Y rows
    f4 sw[2], so;
    // (an 8-wave RCF workgroup: waves 0-3 stage the block)
    const bool stager = !RCF || threadIdx.x < 256;
    if (WST && dphi) stage_slice_lds(a, W, om, fb0, smem);
    if (!WST && dphi && stager) {
      const rsrc_t rw = make_rsrc(W, (int64_t)(RBF ? 2 : 1) * R * g);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int i = (int)threadIdx.x + 256 * j, h = i >= 16 * g, q = i - h * 16 * g;
        const uint32_t off = (uint32_t)((((h * R) + fb0) * g + 4 * q) * 4);
        sw[j] = bload4(rw, i < (RBF ? 32 : 16) * g ? off : DGPRF_OOB);
      }
      const rsrc_t ro = make_rsrc(om, (int64_t)dxw * R);
      const int k = threadIdx.x >> 4, c4 = threadIdx.x & 15;
      so = bload4(ro, k < dxw && fb0 + 4 * c4 < R ? (uint32_t)((k * R + fb0 + 4 * c4) * 4) : DGPRF_OOB);
    }
    STEP_STAMP(stamp_base, 1);
    if (RCF)  // the whole output layer for the F_L recompute, copied while the partials load
      elem_prologue_mid(a, chain, row0, TR * g, xs, dfs, dfst, ysh, red,
                        [&]() { rcf_stage<RBF>(a, W, om, smem); });
    else
      elem_prologue(a, chain, row0, TR * g, xs, dfs, dfst, ysh, red);
    if (!WST && dphi && stager) {
#pragma unroll
      for (int j = 0; j < 2; ++j) *reinterpret_cast<f4*>(wsl + 4 * ((int)threadIdx.x + 256 * j)) = sw[j];
      *reinterpret_cast<f4*>(osl + (threadIdx.x >> 4) * OST + 4 * (threadIdx.x & 15)) = so;
    }
    STEP_STAMP(stamp_base, 4);
  } else {
    if (WST && dphi) stage_slice_lds(a, W, om, fb0, smem);
    if (!WST && dphi) stage_load(fb0);
    if (KS > 0 || !a.a0 || FB) load_x_tile(a, chain, row0, xs);
    for (int e = threadIdx.x; e < TR * g; e += blockDim.x) {  // dF (or F_L) slice sums; Y alongside
      const int r = e / g, o = e - r * g, b = row0 + r, bc = min(b, B - 1);
      const float v = sum_slices((a.last ? fpl : dxn) + (int64_t)bc * g + o, (int64_t)B * g);
      dfs[r * dfst + o] = b < B ? v : 0.f;
      if (a.last) ysh[r * dfst + o] = yr[(int64_t)bc * a.y_cols + min(o, yc - 1)];
    }
  }

  if (RCF) {
    // folded output layer: F_L of this row tile from the X tile (F_{L-1}) and the staged layer,
    // the 4 waves' feature shares summed in wave order into the dF tile (rows >= B: 0)
    __syncthreads();  // X tile, Y values and the LDS copies of W_L / Omega_L
    STEP_STAMP(stamp_base, 5);
    float xr[8];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) xr[ks] = (ks < KS && 4 * ks < d) ? xs[lr * a.xst + 4 * ks + lq] : 0.f;
    const int nw = (int)(blockDim.x >> 6);
    const float v = rcf_row_partial<KS, RBF>(a, smem, xr, cl, wave, nw, lr, lq);
    STEP_STAMP(stamp_base, 7);
    if (lq == 0) red[wave * TR + lr] = v;
    __syncthreads();
    STEP_STAMP(stamp_base, 10);
    if (threadIdx.x < TR) {
      const int r = threadIdx.x;
      float f = red[r];
      for (int w = 1; w < nw; ++w) f += red[w * TR + r];  // wave order
      dfs[r * dfst] = row0 + r < B ? f : 0.f;
    }
    if (threadIdx.x >= 256) return;  // waves 4-7 (no later barrier waits for an ended wave)
  }
  // dF_l tile [16][g]: the last layer turns F_L into the likelihood gradient in place;
  // otherwise dF_l = dX_{l+1}[:, :g_l] (already summed above)
  if (a.last) {
    // likelihood gradient dF = -(1/B) dlogp/dF (likelihoods/gaussian.py:18-25, softmax.py:8-15)
    __syncthreads();
    if (threadIdx.x < TR) {
      const int r = threadIdx.x, b = row0 + r;
      float* df = dfs + r * dfst;
      float lvrow = 0.f;
      if (b < B) {
        const float* y = ysh + r * dfst;
        const float invB = 1.0f / (float)B;
        float logp = 0.f;
        if (a.likelihood == DGPRF_LIK_GAUSSIAN) {
          const float var = a.varptr[(int64_t)chain * a.der_cs];
          const float logvar = logf(var);
          float lv = 0.f;  // d(-log p)/d lik_log_var = sum_o (1 - diff^2/var)/2
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
          // int32(Y[:, 0]) (likelihoods/softmax.py:14); a label outside [0, g) poisons log p and
          // the gradient with NaN instead of scoring a clamped class (TF raises on it)
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
      if (FB && a.lik_fb) {  // the row tile's lik_log_var partial (lanes 0..15, fixed order)
        const float v = sum16(lvrow);
        if (r == 0 && sl == 0) a.hpl[(int64_t)chain * a.ws_cs + rt] = v;
      }
    }
  }
  if (!WST && !a.fast && dphi) stage_store(fb0);
  __syncthreads();
  STEP_STAMP(stamp_base, 2);

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
  // g == 1 operands: dF[row lr] and dF[rows 4lq..4lq+3] in every lane
  const float dg1 = G1 ? dfs[lr * dfst] : 0.f;
  float dg4[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) dg4[r] = G1 ? dfs[(4 * lq + r) * dfst] : 0.f;

  // this row tile's gW partial row, stored write-through (sc1): 13 rows x w_total floats at B = 200
  // that would otherwise sit dirty in the XCD L2s when the launch ends (configs 4 / 5: 12.8 /
  // 13.6 MB per layer; measured config 5 103 -> 98 us/step, config 4 126 -> 124)
  const rsrc_t rgw = make_rsrc(a.gwp + (int64_t)chain * a.ws_cs + (int64_t)rt * a.gw_ld, a.w_cs);
  auto gw_store = [&](int64_t i, float v) { bstore1_wt(v, rgw, (uint32_t)(i * 4)); };
  auto gw_store4 = [&](int64_t i, f4 v) { bstore4_wt(v, rgw, (uint32_t)(i * 4)); };  // i % 4 == 0
  float* gst = smem + a.gst_off + wave * 2 * 16 * g;  // this wave's gW tile staging (g % 16 != 0)
  f4 dxa[NDM];
#pragma unroll
  for (int dt = 0; dt < NDM; ++dt) dxa[dt] = f4zero();
  // full_bayesian=True: per-wave sums over this row tile and the wave's features of
  //   hw[k]     = sum_b X[b][k] (dA z^T)[b][k]   (-> log_inv_ls)
  //   hw[d + k] = sum_b X[b][k] rowsum(dA)[b]    (-> mean)
  //   hw[2d]    = sum dPhi * Phi                  (-> log_amp)
  const int hst = round4(2 * d + 1);
  float* hw = smem + a.hred_off + wave * hst;
  float ampl = 0.f;
  if (FB)
    for (int e = lane; e < hst; e += 64) hw[e] = 0.f;
  for (int i = 0; i < nit; ++i) {
    const int f0 = chunk_f0(i);
    if (f0 >= R) break;
    if (i > 0) {
      if (KS > 0) load_om_frag<KS>(om, R, d, f0, lr, lq, omk);
      if (FB)
#pragma unroll
        for (int dt = 0; dt < NZ; ++dt) zpf[dt] = z_frag(f0, dt);
      if (!WST && dphi) {
        stage_load((sl * cpw + i) * 64);
        __syncthreads();  // every wave is done with the previous block
        stage_store((sl * cpw + i) * 64);
        __syncthreads();
      }
    }
    // ---- phase 1: LDS operands, both A-tile orientations and dPhi (independent chains)
    //   at_t: rows in registers  (gW = Phi^T dF,   K = rows)
    //   at_n: features in registers (dA -> dX = dA Omega^T, K = features)
    //   dPhi = dF W^T in the features-in-registers orientation (K = g)
    float wd0[KGM], wd1[KGM];
    f4 oxv[NDM];
    // this chunk's 64-feature block: the per-chunk staging buffers, or its rows of the slice image
    const float* wsc = WST ? smem + a.wsa_off + i * NWB * 16 * g : wsl;
    const int whalf = WST ? 64 * cpw * g : nwh;
    const float* osc = WST ? smem + a.osa_off + i * NWB * 16 : osl;
    const int ostc = WST ? a.osa_st : OST;
    if (dphi) {
      const bool frow = f0 + lr < R;
#pragma unroll
      for (int ks = 0; ks < KGM; ++ks) {
        const int o = 4 * ks + lq, wo = (wave * 16 + lr) * g + o;
        const bool ok = o < g && frow;
        wd0[ks] = G1 ? 0.f : (ok ? wsc[wo] : 0.f);
        wd1[ks] = (G1 || !RBF) ? 0.f : (ok ? wsc[whalf + wo] : 0.f);
      }
      // rows k >= dxw of the staged block are never written: they only feed discarded outputs
#pragma unroll
      for (int dt = 0; dt < NDM; ++dt)
        oxv[dt] = *reinterpret_cast<const f4*>(osc + (dt * 16 + lr) * ostc + wave * 16 + 4 * lq);
    }
    // layer 0 with d > 32: both orientations read the precomputed A_1 (k_step_agemm)
    const float* a0 = KS == 0 && a.a0 ? a.a0 + (int64_t)chain * a.ws_cs + (int64_t)row0 * R + f0
                                      : nullptr;
    f4 at_t;
    if (KS == 0 && a0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) at_t[r] = a0_sum1(a0 + (int64_t)(4 * lq + r) * R + lr, a.a0_sl);
    } else {
      at_t = a_tile<KS, true>(om, R, d, f0, omk, xf, xs, a.xst, lr, lq);
    }
    f4 at_n = f4zero(), dpc = f4zero(), dps = f4zero();
    if (dphi) {
      at_n = (KS == 0 && a0) ? a0_sum4(a0 + (int64_t)lr * R + 4 * lq, a.a0_sl)
                             : a_tile<KS, false>(om, R, d, f0, omk, xf, xs, a.xst, lr, lq);
      if (G1) {
        // g == 1: dPhi[b][f] = dF[b] W[f] (outer product, VALU)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int fl = wave * 16 + 4 * lq + r;
          const bool ok = f0 + 4 * lq + r < R;
          dpc[r] = ok ? dg1 * wsc[fl] : 0.f;
          dps[r] = (ok && RBF) ? dg1 * wsc[whalf + fl] : 0.f;
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
    // ---- phase 2: transcendentals of both tiles, batched
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
    STEP_STAMP(stamp_base, 8);
    // ---- phase 3: gW_l partial of this row tile, then dX
    if (G1) {
      // g == 1: gW[f] = sum_b Phi[b][f] dF[b]: 4 rows per lane, then across the 4 row groups
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
      const int f = f0 + lr;
      if (lq == 0 && f < R) {
        gw_store(f, gc);
        if (RBF) gw_store(R + f, gs);
      }
    } else {
      // g a multiple of 16 (config 5): dF as the A operand and Phi as B, so the tile comes out as
      // gW^T — a lane holds four consecutive outputs of one feature row and the partial row is
      // written 16 bytes per lane (config 5 94.1 -> 93.0 us/step); other widths keep gW's own
      // orientation and dword stores (16- / 8-byte stores measured slower there: config 2 27.0 ->
      // 27.4, config 4 108.6 -> 121.8 us/step)
      const bool t16 = GSM == 1 || (GSM == 0 && (g & 15) == 0);
      constexpr bool gsv = GSM == 2;
#pragma unroll
      for (int ot = 0; ot < NOT; ++ot) {
        f4 gc = f4zero(), gs = f4zero();
        if (t16) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            gc = mfma16(dfg[ot][r], q0[r], gc);
            if (RBF) gs = mfma16(dfg[ot][r], q1[r], gs);
          }
          // gc[r] = gW[f0 + lr][ot*16 + 4lq + r]
          const int o = ot * 16 + 4 * lq, f = f0 + lr;
          if (f < R) {
            gw_store4((int64_t)f * g + o, gc);
            if (RBF) gw_store4((int64_t)(R + f) * g + o, gs);
          }
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            gc = mfma16(q0[r], dfg[ot][r], gc);
            if (RBF) gs = mfma16(q1[r], dfg[ot][r], gs);
          }
          // gc[r] = gW[f0 + 4lq + r][ot*16 + lr]: to the wave's LDS tile [2][16][g], or stored
          const int o = ot * 16 + lr;
          if (o < g) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int f = f0 + 4 * lq + r;
              if (gsv) {
                gst[(4 * lq + r) * g + o] = gc[r];
                if (RBF) gst[(16 + 4 * lq + r) * g + o] = gs[r];
              } else if (GSM == 0 && f < R) {
                gw_store((int64_t)f * g + o, gc[r]);
                if (RBF) gw_store((int64_t)(R + f) * g + o, gs[r]);
              }
            }
          }
        }
        STEP_STAMP(stamp_base, 9);
      }
      if (gsv) {
        // rows f0 .. f0 + 15 of gW (and of its sin half) are one contiguous run of 16 g floats,
        // written as float4 lanes when every run starts 16-byte aligned (f0 g is a multiple of 16;
        // the sin half starts R g floats on); rows past R are not stored
        __builtin_amdgcn_wave_barrier();
        const int nfl = min(16, R - f0) * g;
        const bool v4 = ((R * g) & 3) == 0 && (nfl & 3) == 0;
#pragma unroll
        for (int h = 0; h < (RBF ? 2 : 1); ++h) {
          const int64_t gb = (int64_t)(h * R + f0) * g;
          const float* src = gst + h * 16 * g;
          if (v4) {
#pragma unroll
            for (int it = 0; it < NOT; ++it) {  // 16 g <= 256 NOT floats: NOT passes of 64 lanes
              const int j = lane + 64 * it;
              if (4 * j < nfl) gw_store4(gb + 4 * j, *reinterpret_cast<const f4*>(src + 4 * j));
            }
          } else {
            for (int j = lane; j < nfl; j += 64) gw_store(gb + j, src[j]);
          }
        }
        __builtin_amdgcn_wave_barrier();
      }
    }
    STEP_STAMP(stamp_base, 6);
    if (dxw > 0) {
#pragma unroll
      for (int dt = 0; dt < NDM; ++dt)
        if (dt < ND) {
#pragma unroll
          for (int r = 0; r < 4; ++r) dxa[dt] = mfma16(oxv[dt][r], da[r], dxa[dt]);
        }
    }
    if (FB) {
      // rowsum(dA) over this chunk: the lane's 4 features, then the 4 feature groups
      float rs = (da[0] + da[1]) + (da[2] + da[3]);
      rs += __shfl_xor(rs, 16);
      rs += __shfl_xor(rs, 32);
      // Dz = dA z^T in 16-dim tiles of the layer input (same contraction as dX with z rows),
      // contracted with the X tile over the 16 rows right away (linear in the features)
      for (int dt = 0; dt * 16 < d; ++dt) {
        f4 zf;
        if (NZ > 0) {
          zf = zpf[0];
#pragma unroll
          for (int q = 1; q < NZ; ++q)
            if (dt == q) zf = zpf[q];
        } else {
          zf = z_frag(f0, dt);
        }
        f4 dz = f4zero();
#pragma unroll
        for (int r = 0; r < 4; ++r) dz = mfma16(zf[r], da[r], dz);
        // dz[r] = Dz[row lr][dt*16 + 4lq + r]
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int kk = dt * 16 + 4 * lq + r;
          const float xv = kk < d ? xs[lr * a.xst + kk] : 0.f;
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
  STEP_STAMP(stamp_base, 3);
  if (FB) {
    // log_amp term over the wave, then the workgroup's partial row [2d+1] in wave order
    float v = sum16(ampl);
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    if (lane == 0) hw[2 * d] = v;
    __syncthreads();
    float* hp = a.hp + (int64_t)chain * a.ws_cs + ((int64_t)rt * NSM + sl) * hst;
    const float* h0 = smem + a.hred_off;
    for (int e = threadIdx.x; e < 2 * d + 1; e += blockDim.x)
      hp[e] = ((h0[e] + h0[hst + e]) + h0[2 * hst + e]) + h0[3 * hst + e];  // FB: NWB == 4
  }
  if (dxw > 0) {
    // dxa[dt][r] = dX[row lr][dt*16 + 4lq + r]; sum the 4 waves in LDS, store the slice partial.
    // row stride DPS = 16 ND + 4: conflict-free 16-byte row writes (as the forward's F rows)
    const int DPS = ND * 16 + 4;
    float* redw = red + wave * TR * DPS;
#pragma unroll
    for (int dt = 0; dt < NDM; ++dt)
      if (dt < ND) *reinterpret_cast<f4*>(redw + lr * DPS + dt * 16 + 4 * lq) = dxa[dt];
    __syncthreads();
    float* dxp = a.dxout + (int64_t)chain * a.ws_cs + (int64_t)sl * B * dxw;
    // write-through (sc1), as the forward's F partials
    const rsrc_t rdx = make_rsrc(dxp, (int64_t)B * dxw);
    for (int e = threadIdx.x; e < TR * dxw; e += blockDim.x) {
      const int r = e / dxw, k = e - r * dxw, b = row0 + r;
      if (b < B) {
        float v = red[r * DPS + k];
#pragma unroll
        for (int w = 1; w < NWB; ++w) v += red[w * TR * DPS + r * DPS + k];
        bstore1_wt(v, rdx, (uint32_t)(((int64_t)b * dxw + k) * 4));
      }
    }
  }
#ifdef DGPRF_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  STEP_STAMP(stamp_base, 14);
}

// backward: KS x NOT x RBF x G1 x FB x waves per workgroup (8: W-only with whole-slice staging)
// the 8-wave (whole-slice) instances fix the gW store form at compile time: transposed tile for
// g % 16 == 0 (and g == 1, which uses neither), LDS-staged otherwise (make_layer_k reserves the
// staging whenever it keeps the whole-slice layout)
// the folded output layer's workgroup: 8 waves when R % 512 == 0 (every wave's chunks in groups of
// 4), 4 otherwise (R % 256 == 0, step_fold_out)
inline int rcf_threads(const LayerK& a) {
#ifdef DGPRF_RCF4
  return 256;
#else
  return a.R % 512 == 0 ? 512 : 256;
#endif
}
template <int KS, int NOT, bool G1>
void k_step_bwd_launch3(bool rbf, bool fb, bool w8, bool t16, dim3 grid, size_t lds,
                        hipStream_t s, const LayerK& a) {
#define DGPRF_BWD(R_, F_, W_, M_)                                                                  \
  do {                                                                                            \
    dgprf::set_lds_limit((const void*)k_step_bwd<KS, NOT, R_, G1, F_, W_, M_>, lds);             \
    hipLaunchKernelGGL((k_step_bwd<KS, NOT, R_, G1, F_, W_, M_>), grid, dim3(64 * W_), lds, s, a); \
  } while (0)
  constexpr int GS = G1 ? 1 : 2;
  if constexpr (G1 && KS > 0) {
    if (a.rcf) {  // folded output layer (make_layer_k sets rcf only for 4-wave W-only launches)
      if (rbf) {
        dgprf::set_lds_limit((const void*)k_step_bwd<KS, NOT, true, G1, false, 4, 0, true>, lds);
        hipLaunchKernelGGL((k_step_bwd<KS, NOT, true, G1, false, 4, 0, true>), grid, dim3(rcf_threads(a)), lds, s, a);
      } else {
        dgprf::set_lds_limit((const void*)k_step_bwd<KS, NOT, false, G1, false, 4, 0, true>, lds);
        hipLaunchKernelGGL((k_step_bwd<KS, NOT, false, G1, false, 4, 0, true>), grid, dim3(rcf_threads(a)), lds, s, a);
      }
      return;
    }
  }
  if (rbf) {
    if (fb) DGPRF_BWD(true, true, 4, 0);
    else if (w8 && t16) DGPRF_BWD(true, false, 8, 1);
    else if (w8) DGPRF_BWD(true, false, 8, GS);
    else DGPRF_BWD(true, false, 4, 0);
  } else {
    if (fb) DGPRF_BWD(false, true, 4, 0);
    else if (w8 && t16) DGPRF_BWD(false, false, 8, 1);
    else if (w8) DGPRF_BWD(false, false, 8, GS);
    else DGPRF_BWD(false, false, 4, 0);
  }
#undef DGPRF_BWD
}
template <int KS>
void k_step_bwd_launch2(int g, bool rbf, bool fb, bool w8, dim3 grid, size_t lds, hipStream_t s,
                        const LayerK& a) {
  const int NOT = (g + 15) >> 4;
  const bool t16 = (g & 15) == 0;
  if (g == 1) k_step_bwd_launch3<KS, 1, true>(rbf, fb, w8, t16, grid, lds, s, a);
  else if (NOT == 1) k_step_bwd_launch3<KS, 1, false>(rbf, fb, w8, t16, grid, lds, s, a);
  else if (NOT == 2) k_step_bwd_launch3<KS, 2, false>(rbf, fb, w8, t16, grid, lds, s, a);
  else if (NOT == 3) k_step_bwd_launch3<KS, 3, false>(rbf, fb, w8, t16, grid, lds, s, a);
  else k_step_bwd_launch3<KS, 4, false>(rbf, fb, w8, t16, grid, lds, s, a);
}

}  // namespace dgprf_sk

#ifdef DGPRF_KS
template void dgprf_sk::k_step_bwd_launch2<DGPRF_KS>(int, bool, bool, bool, dim3, size_t,
                                                       hipStream_t, const dgprf_sk::LayerK&);
#endif
