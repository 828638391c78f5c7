// step_fwd_impl.h — the step forward kernel k_step_fwd (one layer of BNN_from_list.__call__,
// utils.py:10-44: Omega x -> c [cos|sin] or c relu -> Phi W, layers/rf_layers.py:29-45,75-91,
// layers/GP_weight_layers.py:11-15) and its launch dispatch, included by step_fwd_k<KS>.hip.
#pragma once
#include "step_common.h"

namespace dgprf_sk {

template <int KS, int NOT, bool RBF, bool G1, int NWB>
__global__ __launch_bounds__(64 * NWB) void k_step_fwd(const LayerK a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  int rt, sl;
  if (!tile_of_block(a, rt, sl)) return;
  const int chain = blockIdx.z;
  const float* __restrict__ om = a.om + (int64_t)chain * a.om_cs;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, lr = lane & 15, lq = lane >> 4;
  const int R = a.R, g = a.g, d = a.d, B = a.B, cpw = a.cpw;
  const int row0 = rt * TR;
  const int stamp_base = (a.layer * 2) * 4096 + blockIdx.z * gridDim.x + blockIdx.x;
  STEP_STAMP(stamp_base, 0);
  float* xs = smem;
  float* red = smem + a.red_off;
  const float* __restrict__ W = a.W + (int64_t)chain * a.w_cs;
  // the slice's 4 cpw 16-feature chunks: iteration i of wave w takes chunk i NWB + w
  auto chunk_f0 = [&](int i) { return ((sl * cpw * 4 + i * NWB) + wave) * 16; };
  const int nit = cpw * 4 / NWB;

  // first chunk's fragments: independent of the X tile, issued first
  float omk[8], wf[NOT][4][2];
  if (KS > 0) load_om_frag<KS>(om, R, d, chunk_f0(0), lr, lq, omk);
  load_w_frag<NOT, RBF, G1>(W, R, g, chunk_f0(0), lr, lq, wf);
  const float cl = a.cptr[(int64_t)chain * a.der_cs];
  STEP_STAMP(stamp_base, 1);
  if (a.fast) {
    elem_prologue(a, chain, row0, 0, xs, red, 0, red, red);  // no dF tile: unused targets
  } else if (KS > 0 || !a.a0) {
    load_x_tile(a, chain, row0, xs);
  }
  const float* a0 = KS == 0 && a.a0 ? a.a0 + (int64_t)chain * a.ws_cs + (int64_t)(row0 + lr) * R : nullptr;
  __syncthreads();
  STEP_STAMP(stamp_base, 2);

  float xf[8];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) xf[ks] = (ks < KS && 4 * ks < d) ? xs[lr * a.xst + 4 * ks + lq] : 0.f;

  f4 acc[NOT], acs[NOT];
#pragma unroll
  for (int ot = 0; ot < NOT; ++ot) acc[ot] = acs[ot] = f4zero();
  float acc1 = 0.f;  // G1: per-lane partial of F[row lr]
  STEP_STAMP(stamp_base, 6);
  for (int i = 0; i < nit; ++i) {
    const int f0 = chunk_f0(i);
    if (f0 >= R) break;
    const f4 at = (KS == 0 && a0) ? a0_sum4(a0 + f0 + 4 * lq, a.a0_sl)
                                  : a_tile<KS, false>(om, R, d, f0, omk, xf, xs, a.xst, lr, lq);
    float p0[4], p1[4];
    features<RBF>(at, cl, p0, p1);
    float wc[NOT][4][2];
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool ok = w_ok<G1>(ot, r, R, g, f0, lr, lq);
        wc[ot][r][0] = keep(wf[ot][r][0], ok);
        wc[ot][r][1] = keep(wf[ot][r][1], ok);
      }
    if (i + 1 < nit) {  // prefetch the next chunk (clamped loads are always in range)
      if (KS > 0) load_om_frag<KS>(om, R, d, chunk_f0(i + 1), lr, lq, omk);
      load_w_frag<NOT, RBF, G1>(W, R, g, chunk_f0(i + 1), lr, lq, wf);
    }
    if (G1) {
      // g == 1: F[row lr] += sum_f Phi[lr][f] W[f], 4 features per lane (VALU)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        acc1 = fmaf(p0[r], wc[0][r][0], acc1);
        if (RBF) acc1 = fmaf(p1[r], wc[0][r][1], acc1);
      }
    } else {
#pragma unroll
      for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          acc[ot] = mfma16(wc[ot][r][0], p0[r], acc[ot]);
          if (RBF) acs[ot] = mfma16(wc[ot][r][1], p1[r], acs[ot]);
        }
    }
  }
  STEP_STAMP(stamp_base, 7);
  // acc[ot][r] = F[row lr][ot*16 + 4lq + r]; sum the 4 waves' feature chunks in LDS.  Row stride
  // GPS = 16 NOT + 4: the 16-byte row writes of 8 lanes (one LDS cycle group) start 4 banks apart
  // (a stride of 16 NOT put all 16 rows on one bank: 16-way conflicts)
  constexpr int GPS = NOT * 16 + 4;
  float* redw = red + wave * TR * GPS;
  if (G1) {
    acc1 += __shfl_xor(acc1, 16);
    acc1 += __shfl_xor(acc1, 32);
    if (lq == 0) redw[lr * GPS] = acc1;
  } else {
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot)
      *reinterpret_cast<f4*>(redw + lr * GPS + ot * 16 + 4 * lq) = acc[ot] + acs[ot];
  }
  STEP_STAMP(stamp_base, 3);
  __syncthreads();
  float* fp = a.fout + (int64_t)chain * a.ws_cs + (int64_t)sl * B * g;
  // slice partials stored write-through (sc1), like the gW partials: nothing of them is left dirty
  // in the L2 for the launch boundary to write back (config 3 35.4 -> 35.0 us/step, others level)
  const rsrc_t rfp = make_rsrc(fp, (int64_t)B * g);
  for (int e = threadIdx.x; e < TR * g; e += blockDim.x) {
    const int r = e / g, o = e - r * g, b = row0 + r;
    if (b < B) {
      float v = red[r * GPS + o];
#pragma unroll
      for (int w = 1; w < NWB; ++w) v += red[w * TR * GPS + r * GPS + o];
      bstore1_wt(v, rfp, (uint32_t)(((int64_t)b * g + o) * 4));
    }
  }
#ifdef DGPRF_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  STEP_STAMP(stamp_base, 14);
}

// forward: KS x NOT x RBF x G1 x waves per workgroup (8 / 16 for slices of >= 2 chunks per wave:
// two / four waves per SIMD hide each other's MFMA / load latency; 4 otherwise)
template <int KS, int NOT, bool G1>
void k_step_fwd_launch3(bool rbf, int nw, dim3 grid, size_t lds, hipStream_t s, const LayerK& a) {
#define DGPRF_FWD(R_, W_)                                                                  \
  do {                                                                                    \
    dgprf::set_lds_limit((const void*)k_step_fwd<KS, NOT, R_, G1, W_>, lds);             \
    hipLaunchKernelGGL((k_step_fwd<KS, NOT, R_, G1, W_>), grid, dim3(64 * W_), lds, s, a); \
  } while (0)
  if (nw == 16) {
    if (rbf) DGPRF_FWD(true, 16);
    else DGPRF_FWD(false, 16);
  } else if (nw == 8) {
    if (rbf) DGPRF_FWD(true, 8);
    else DGPRF_FWD(false, 8);
  } else {
    if (rbf) DGPRF_FWD(true, 4);
    else DGPRF_FWD(false, 4);
  }
#undef DGPRF_FWD
}
template <int KS>
void k_step_fwd_launch2(int g, bool rbf, int nw, dim3 grid, size_t lds, hipStream_t s,
                        const LayerK& a) {
  const int NOT = (g + 15) >> 4;
  if (g == 1) k_step_fwd_launch3<KS, 1, true>(rbf, nw, grid, lds, s, a);
  else if (NOT == 1) k_step_fwd_launch3<KS, 1, false>(rbf, nw, grid, lds, s, a);
  else if (NOT == 2) k_step_fwd_launch3<KS, 2, false>(rbf, nw, grid, lds, s, a);
  else if (NOT == 3) k_step_fwd_launch3<KS, 3, false>(rbf, nw, grid, lds, s, a);
  else k_step_fwd_launch3<KS, 4, false>(rbf, nw, grid, lds, s, a);
}

}  // namespace dgprf_sk

// one translation unit per KS: #define DGPRF_KS before including this header
#ifdef DGPRF_KS
template void dgprf_sk::k_step_fwd_launch2<DGPRF_KS>(int, bool, int, dim3, size_t, hipStream_t,
                                                       const dgprf_sk::LayerK&);
#endif
