// agemm.hip — A_1 = X Omega_1 for a wide first layer (d_1 > 32, e.g. the 784 MNIST pixels of
// BASELINE config 4): the `tf.matmul(x, self.Omega)` of RBFLayer / ARCLayer
// (layers/rf_layers.py:42, 88) as one hand-written fp32 MFMA GEMM, A[n][R] = X[n][d] Omega[d][R],
// all row-major, for the step (n = B rows, ~200) and the predictive forward (row chunks of the test
// set, ~10k rows).
//
// v_mfma_f32_32x32x2_f32 (exact fp32 fma chain, 64 cycles issue = dependent latency, so one
// accumulator chain per wave already runs at the MFMA rate).  A workgroup of 4 waves computes a
// BM x BN tile; wave w owns a WM x WN sub-tile of (WM / 32) x (WN / 32) accumulators.  K runs in
// LDS-staged blocks of BK = 32: the next block's X / Omega tiles are loaded into registers (16-byte
// loads) while the current block's 16 k-steps run, then written to the other LDS buffer — one
// barrier per block.  LDS images: X as [BK][BM + 1] (k-major: the A fragment of a k-step is 32
// consecutive rows of one k, conflict-free; the +1 spreads the transposing writes over the banks)
// and Omega as [BK][BN] (its natural row layout).  Rows >= n, k >= d and columns >= R stage as
// zeros; rows [n, n_out) of the output are written as zeros (the step's A_1 buffer is
// [align32(B)][R] and its consumers read whole 16-row tiles).
//
// Tiles: the step (n_out <= 1024 rows, B = 200 -> 224) runs 64 x 64 tiles in two K parts
// (blockIdx.y = chain * 2 + part, part p -> output slab p, summed by the consumers, k_step_fwd /
// k_step_bwd layer 0, as slab 0 + slab 1): 4 x 64 x 2 = 512 workgroups, two per CU, so one
// workgroup's barrier and load waits overlap the other's MFMAs (one 32 x 128 tile per CU, K whole,
// ran 24.5 us; 64 x 64 in two parts 20.6 us — scripts/microbench/agemm_variants.hip).  The step
// tiles are dealt XCD-contiguously (workgroup b runs on XCD b % 8: XCD x takes tiles
// [x G / 8, (x + 1) G / 8), row tile fastest), so each XCD's L2 holds the Omega column blocks of all
// of its row tiles; the next k-step's LDS operands are read ahead of this k-step's MFMAs
// (sched_group_barrier).  Larger n (predictive chunks, ~10k rows): 128 x 128 tiles (64 x 64 per
// wave), K whole, blockIdx order (79 x 32 = 2,528 workgroups).
#include "dgprf_internal.h"

namespace {

typedef float f16v __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f16v mfma32(float a, float b, f16v c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

constexpr int AG_BK = 32;

struct AgArgs {
  const float* X;   // [n][ldx] of batch 0 (batch stride sx)
  const float* om;  // [d][R] of batch 0 (batch stride so; 0 = shared)
  float* out;       // [n_out][R] of batch 0 (batch stride sa); K part p at + p * sp
  int64_t sx, so, sa, sp;
  int32_t n, n_out, ldx, d, R, n_mt;
};

// Workgroup b of G: XCD-contiguous tile order (XCD = b % 8 under round-robin dispatch; a pure speed
// choice — any placement gives the same result), row tile fastest within an XCD's range.
__device__ __forceinline__ void ag_tile(int b, int G, int n_mt, bool xcd, int& mt, int& nt) {
  int L = b;
  if (xcd) {
    const int x = b & 7, j = b >> 3, q = G >> 3, r = G & 7;
    L = x < r ? x * (q + 1) + j : r * (q + 1) + (x - r) * q + j;
  }
  mt = L % n_mt;
  nt = L / n_mt;
}

// SK: K parts (blockIdx.y = batch * SK + part); SCHED: the next k-step's LDS reads are issued ahead
// of this k-step's MFMAs (two register sets); XCD: ag_tile's XCD-contiguous order.
template <int BM, int BN, int WM, int WN, int SK, bool SCHED, bool XCD>
__global__ __launch_bounds__(256) void k_agemm(const AgArgs a) {
  static_assert((BM / WM) * (BN / WN) == 4, "4 waves per workgroup");
  constexpr int MT = WM / 32, NT = WN / 32;            // accumulator tiles per wave
  constexpr int AST = BM + 1;                          // X image row stride (k-major)
  constexpr int A4 = BM * AG_BK / 4 / 256;             // float4 of X per thread per block
  constexpr int B4 = BN * AG_BK / 4 / 256;             // float4 of Omega per thread per block
  static_assert(A4 >= 1 && B4 >= 1, "tile too small for 256 threads");
  __shared__ float As[2][AG_BK * AST];
  __shared__ __attribute__((aligned(16))) float Bs[2][AG_BK * BN];
  int mt, ntile;
  ag_tile(blockIdx.x, gridDim.x, a.n_mt, XCD, mt, ntile);
  const int m0 = mt * BM, n0 = ntile * BN;
  const int64_t bz = blockIdx.y / SK;
  const int part = SK > 1 ? (int)(blockIdx.y % SK) : 0;
  const float* X = a.X + bz * a.sx;
  const float* om = a.om + bz * a.so;
  float* out = a.out + bz * a.sa + part * a.sp;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wr = wave / (BN / WN), wc = wave % (BN / WN);
  const int n = a.n, d = a.d, R = a.R, ldx = a.ldx;
  const rsrc_t rx = make_rsrc(X, (int64_t)n * ldx);
  const rsrc_t ro = make_rsrc(om, (int64_t)d * R);

  f4 xa[A4], ob[B4];
  // thread's staging elements: X float4 q = tid + 256 j -> row q / (BK/4), k4 q % (BK/4);
  // Omega float4 q -> k row q / (BN/4), column 4 (q % (BN/4))
  auto load = [&](int k0) {
#pragma unroll
    for (int j = 0; j < A4; ++j) {
      const int q = tid + 256 * j, r = q / (AG_BK / 4), k = k0 + 4 * (q % (AG_BK / 4));
      const int row = m0 + r;
      // d % 4 == 0 (host-checked), so a float4 never straddles the k edge
      xa[j] = bload4(rx, row < n && k < d ? (uint32_t)(((int64_t)row * ldx + k) * 4) : DGPRF_OOB);
    }
#pragma unroll
    for (int j = 0; j < B4; ++j) {
      const int q = tid + 256 * j, k = k0 + q / (BN / 4), c = n0 + 4 * (q % (BN / 4));
      ob[j] = bload4(ro, k < d && c < R ? (uint32_t)(((int64_t)k * R + c) * 4) : DGPRF_OOB);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < A4; ++j) {
      const int q = tid + 256 * j, r = q / (AG_BK / 4), k = 4 * (q % (AG_BK / 4));
#pragma unroll
      for (int c = 0; c < 4; ++c) As[buf][(k + c) * AST + r] = xa[j][c];
    }
#pragma unroll
    for (int j = 0; j < B4; ++j) {
      const int q = tid + 256 * j, k = q / (BN / 4), c = 4 * (q % (BN / 4));
      *reinterpret_cast<f4*>(&Bs[buf][k * BN + c]) = ob[j];
    }
  };

  f16v acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // K part `part`: k-blocks [kb0, kb0 + nkb) (a part past d stages zeros and writes zeros)
  const int nkb_all = (d + AG_BK - 1) / AG_BK, per = (nkb_all + SK - 1) / SK;
  const int kb0 = part * per, nkb = max(0, min(per, nkb_all - kb0));
  load(kb0 * AG_BK);
  store(0);
  __syncthreads();
  const int li = lane & 31, lk = lane >> 5;  // A[i][k] / B[k][j] operand lane map of 32x32x2
  for (int kb = 0; kb < nkb; ++kb) {
    const int buf = kb & 1;
    if (kb + 1 < nkb) load((kb0 + kb + 1) * AG_BK);
    const float* ap = &As[buf][lk * AST + wr * WM + li];
    const float* bp = &Bs[buf][lk * BN + wc * WN + li];
    if (SCHED) {
      float av[2][MT], bv[2][NT];
#pragma unroll
      for (int i = 0; i < MT; ++i) av[0][i] = ap[32 * i];
#pragma unroll
      for (int j = 0; j < NT; ++j) bv[0][j] = bp[32 * j];
#pragma unroll
      for (int ks = 0; ks < AG_BK / 2; ++ks) {
        const int c = ks & 1;
        if (ks + 1 < AG_BK / 2) {
#pragma unroll
          for (int i = 0; i < MT; ++i) av[c ^ 1][i] = ap[2 * (ks + 1) * AST + 32 * i];
#pragma unroll
          for (int j = 0; j < NT; ++j) bv[c ^ 1][j] = bp[2 * (ks + 1) * BN + 32 * j];
        }
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NT; ++j) acc[i][j] = mfma32(av[c][i], bv[c][j], acc[i][j]);
        // the scheduler otherwise sinks the reads below the MFMAs (one register set, every k-step
        // waiting on its own reads): reads of ks + 1 first, then the MFMAs of ks
        if (ks + 1 < AG_BK / 2) __builtin_amdgcn_sched_group_barrier(0x100, MT + NT, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, MT * NT, 0);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < AG_BK / 2; ++ks) {
        float av[MT], bv[NT];
#pragma unroll
        for (int i = 0; i < MT; ++i) av[i] = ap[2 * ks * AST + 32 * i];
#pragma unroll
        for (int j = 0; j < NT; ++j) bv[j] = bp[2 * ks * BN + 32 * j];
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NT; ++j) acc[i][j] = mfma32(av[i], bv[j], acc[i][j]);
      }
    }
    if (kb + 1 < nkb) store(buf ^ 1);
    __syncthreads();
  }
  // D[row (r & 3) + 8 (r >> 2) + 4 (lane >> 5)][col lane & 31] of each 32 x 32 accumulator
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int col = n0 + wc * WN + 32 * j + li;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wr * WM + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (row < a.n_out && col < R) out[(int64_t)row * R + col] = row < n ? acc[i][j][r] : 0.f;
      }
    }
}

template <int BM, int BN, int WM, int WN, int SK, bool SCHED, bool XCD>
hipError_t agemm_launch(AgArgs a, int batch, hipStream_t s) {
  a.n_mt = (a.n_out + BM - 1) / BM;
  const int n_nt = (a.R + BN - 1) / BN;
  dim3 grid((unsigned)(a.n_mt * n_nt), (unsigned)(batch * SK));
  hipLaunchKernelGGL((k_agemm<BM, BN, WM, WN, SK, SCHED, XCD>), grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace

namespace dgprf {

bool agemm_shape_ok(int64_t n, int64_t n_out, int ldx, int d, int R) {
  return n >= 1 && n_out >= n && d % 4 == 0 && ldx % 4 == 0 && R % 4 == 0 &&
         n_out * (int64_t)R < ((int64_t)1 << 31) && n * (int64_t)ldx < ((int64_t)1 << 29) &&
         (int64_t)d * R < ((int64_t)1 << 29);
}

int agemm_parts(int64_t n, int64_t n_out, int ldx, int d, int R) {
  return agemm_shape_ok(n, n_out, ldx, d, R) && n_out <= 1024 ? 2 : 1;
}

// false: the shape is outside this kernel (the caller falls back to k_step_agemm).  parts = 2
// (only as agemm_parts returns it): two K-part slabs sp floats apart, for consumers that sum them.
bool own_agemm(const float* X, int64_t n, int64_t n_out, int ldx, int d, const float* om, int R,
               float* aout, int batch, int64_t sx, int64_t so, int64_t sa, int parts, int64_t sp,
               hipStream_t s, hipError_t* err) {
  if (!agemm_shape_ok(n, n_out, ldx, d, R)) return false;
  if (parts != 1 && parts != agemm_parts(n, n_out, ldx, d, R)) {
    *err = hipErrorInvalidValue;
    return true;
  }
  AgArgs a;
  a.X = X;
  a.om = om;
  a.out = aout;
  a.sx = sx;
  a.so = so;
  a.sa = sa;
  a.sp = sp;
  a.n = (int32_t)n;
  a.n_out = (int32_t)n_out;
  a.ldx = ldx;
  a.d = d;
  a.R = R;
  a.n_mt = 0;
  // step-sized row counts: 64 x 64 tiles (K whole, or two parts); otherwise 128 x 128
  if (parts == 2) *err = agemm_launch<64, 64, 32, 32, 2, true, true>(a, batch, s);
  else if (n_out <= 1024) *err = agemm_launch<64, 64, 32, 32, 1, true, true>(a, batch, s);
  else *err = agemm_launch<128, 128, 64, 64, 1, false, false>(a, batch, s);
  return true;
}

}  // namespace dgprf
