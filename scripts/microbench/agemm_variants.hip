// agemm_variants.hip — diagnostic microbenchmark of A_1 = X Omega_1 GEMM variants (fp32 MFMA) on
// config 4's two shapes: the step (200 rows -> 224 padded x 784 x 4096) and a predictive chunk
// (10,000 x 784 x 4096).  Each variant is checked against a float64 host reference on sampled
// outputs and timed with hipEvents over back-to-back launches.  Not product code.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o agemm_variants agemm_variants.hip
//   ./agemm_variants
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../../dgp-rf-mcmc_amd/csrc/dgprf_device.h"

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef float f16v __attribute__((ext_vector_type(16)));

struct Args {
  const float* X;
  const float* om;
  float* out;
  int n, n_out, ldx, d, R, n_mt;
  int gm;  // 0: tile = blockIdx (row tile fastest); > 0: XCD-aware order, groups of gm row tiles
  int ksplit;  // k_v1: K parts over blockIdx.y, part p into output slab p
};

// Workgroup b of G runs on XCD b % 8 (round-robin dispatch).  XCD-aware: XCD x takes a contiguous
// range of logical tiles, walked in groups of gm row tiles (row tile fastest inside a group), so the
// row and column blocks its concurrent workgroups share stay in its own L2.
__device__ __forceinline__ void tile_of(const Args& a, int b, int G, int& mt, int& nt) {
  int L = b;
  if (a.gm > 0) {
    const int x = b & 7, j = b >> 3, q = G >> 3, r = G & 7;
    L = x < r ? x * (q + 1) + j : r * (q + 1) + (x - r) * q + j;
    const int n_nt = G / a.n_mt;  // (grid = n_mt * n_nt)
    const int per = a.gm * n_nt, grp = L / per, in = L % per;
    const int rows = min(a.gm, a.n_mt - grp * a.gm);
    mt = grp * a.gm + in % rows;
    nt = in / rows;
    return;
  }
  mt = L % a.n_mt;
  nt = L / a.n_mt;
}

// ---------------------------------------------------------------- V1: the shipped kernel shape
// 32x32x2, X staged transposed [BK][BM+1], Omega [BK][BN], register-staged double buffer.
template <int BM, int BN, int WM, int WN, int PF, int EPI = 0>
__global__ __launch_bounds__(256) void k_v1(const Args a) {
  constexpr int BK = 32;
  constexpr int MT = WM / 32, NT = WN / 32;
  constexpr int AST = BM + 1;
  constexpr int A4 = BM * BK / 4 / 256, B4 = BN * BK / 4 / 256;
  __shared__ float As[2][BK * AST];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK * BN];
  int mt, ntile;
  tile_of(a, blockIdx.x, gridDim.x, mt, ntile);
  const int m0 = mt * BM, n0 = ntile * BN;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wr = wave / (BN / WN), wc = wave % (BN / WN);
  const rsrc_t rx = make_rsrc(a.X, (int64_t)a.n * a.ldx);
  const rsrc_t ro = make_rsrc(a.om, (int64_t)a.d * a.R);
  f4 xa[A4], ob[B4];
  auto load = [&](int k0) {
#pragma unroll
    for (int j = 0; j < A4; ++j) {
      const int q = tid + 256 * j, r = q / (BK / 4), k = k0 + 4 * (q % (BK / 4)), row = m0 + r;
      xa[j] = bload4(rx, row < a.n && k < a.d ? (uint32_t)(((int64_t)row * a.ldx + k) * 4) : DGPRF_OOB);
    }
#pragma unroll
    for (int j = 0; j < B4; ++j) {
      const int q = tid + 256 * j, k = k0 + q / (BN / 4), c = n0 + 4 * (q % (BN / 4));
      ob[j] = bload4(ro, k < a.d && c < a.R ? (uint32_t)(((int64_t)k * a.R + c) * 4) : DGPRF_OOB);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < A4; ++j) {
      const int q = tid + 256 * j, r = q / (BK / 4), k = 4 * (q % (BK / 4));
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
  const int nkb_all = (a.d + BK - 1) / BK, per = (nkb_all + a.ksplit - 1) / a.ksplit;
  const int kb0 = blockIdx.y * per, nkb = min(per, nkb_all - kb0);
  float* out = a.out + (size_t)blockIdx.y * a.n_out * a.R;
  load(kb0 * BK);
  store(0);
  __syncthreads();
  const int li = lane & 31, lk = lane >> 5;
  for (int kb = 0; kb < nkb; ++kb) {
    const int buf = kb & 1;
    if (kb + 1 < nkb) load((kb0 + kb + 1) * BK);
    const float* ap = &As[buf][lk * AST + wr * WM + li];
    const float* bp = &Bs[buf][lk * BN + wc * WN + li];
    if (PF == 0) {
#pragma unroll
      for (int ks = 0; ks < BK / 2; ++ks) {
        float av[MT], bv[NT];
#pragma unroll
        for (int i = 0; i < MT; ++i) av[i] = ap[2 * ks * AST + 32 * i];
#pragma unroll
        for (int j = 0; j < NT; ++j) bv[j] = bp[2 * ks * BN + 32 * j];
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NT; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);
      }
    } else if (PF == 1 || PF == 3) {
      float av[2][MT], bv[2][NT];
#pragma unroll
      for (int i = 0; i < MT; ++i) av[0][i] = ap[32 * i];
#pragma unroll
      for (int j = 0; j < NT; ++j) bv[0][j] = bp[32 * j];
#pragma unroll
      for (int ks = 0; ks < BK / 2; ++ks) {
        const int c = ks & 1;
        if (ks + 1 < BK / 2) {
#pragma unroll
          for (int i = 0; i < MT; ++i) av[c ^ 1][i] = ap[2 * (ks + 1) * AST + 32 * i];
#pragma unroll
          for (int j = 0; j < NT; ++j) bv[c ^ 1][j] = bp[2 * (ks + 1) * BN + 32 * j];
        }
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NT; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[c][i], bv[c][j], acc[i][j], 0, 0, 0);
        if (PF == 3) {  // next k-step's reads ahead of this one's MFMAs
          if (ks + 1 < BK / 2) __builtin_amdgcn_sched_group_barrier(0x100, MT + NT, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, MT * NT, 0);
        }
      }
    } else {
      float av[BK / 2][MT], bv[BK / 2][NT];
#pragma unroll
      for (int ks = 0; ks < BK / 2; ++ks) {
#pragma unroll
        for (int i = 0; i < MT; ++i) av[ks][i] = ap[2 * ks * AST + 32 * i];
#pragma unroll
        for (int j = 0; j < NT; ++j) bv[ks][j] = bp[2 * ks * BN + 32 * j];
      }
#pragma unroll
      for (int ks = 0; ks < BK / 2; ++ks)
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NT; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[ks][i], bv[ks][j], acc[i][j], 0, 0, 0);
    }
    if (kb + 1 < nkb) store(buf ^ 1);
    __syncthreads();
  }
  if (EPI) {  // accumulators -> LDS (per wave [WM][WN + 4]) -> 16-byte row stores
    constexpr int EST = WN;  // (the two lane halves of a ds_write_b32 are separate bank groups)
    static_assert(4 * WM * EST <= 2 * BK * (AST + BN), "epilogue staging");
    float* eb = &As[0][0] + wave * WM * EST;  // As and Bs are contiguous
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          eb[(32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk) * EST + 32 * j + li] = acc[i][j][r];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): own wave's writes (wave-private region)
#pragma unroll
    for (int e = lane; e < WM * WN / 4; e += 64) {
      const int rr = e / (WN / 4), c4 = e % (WN / 4);
      const int row = m0 + wr * WM + rr, col = n0 + wc * WN + 4 * c4;
      const f4 v = *reinterpret_cast<const f4*>(eb + rr * EST + 4 * c4);
      if (row < a.n_out && col < a.R)
        *reinterpret_cast<f4*>(out + (int64_t)row * a.R + col) = row < a.n ? v : f4{0.f, 0.f, 0.f, 0.f};
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int col = n0 + wc * WN + 32 * j + li;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wr * WM + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (row < a.n_out && col < a.R) out[(int64_t)row * a.R + col] = row < a.n ? acc[i][j][r] : 0.f;
      }
    }
}

// ---------------------------------------------------------------- V2: 16x16x4, no transposition
// X staged k-quad-major [BK/4][BM][4] (one ds_write_b128 per float4, conflict-free A reads:
// lane (i, kq) reads element kq of row i's quad), Omega [BK][BN+16] (the +16 row pad puts the
// four k rows of a B read in four bank groups).  KS wave groups split the k-blocks (group g runs
// blocks g, g + KS, ...) with their own LDS buffers; their accumulators are summed in LDS at the
// end in group order.  NB: LDS buffers per group (2 = double buffer).
template <int BM, int BN, int WM, int WN, int KS, int BK>
__global__ __launch_bounds__(64 * (BM / WM) * (BN / WN) * KS) void k_v2(const Args a) {
  constexpr int WPG = (BM / WM) * (BN / WN);  // waves per k group
  constexpr int TPG = 64 * WPG;
  constexpr int MT = WM / 16, NT = WN / 16;
  constexpr int BST = BN + 16;
  constexpr int ASZ = BK * BM, BSZ = BK * BST;
  constexpr int A4 = (BM * BK / 4 + TPG - 1) / TPG, B4 = (BN * BK / 4 + TPG - 1) / TPG;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  int mt, ntile;
  tile_of(a, blockIdx.x, gridDim.x, mt, ntile);
  const int m0 = mt * BM, n0 = ntile * BN;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 15, lq = lane >> 4;
  const int grp = wave / WPG, gw = wave % WPG, gt = tid - grp * TPG;
  const int wr = gw / (BN / WN), wc = gw % (BN / WN);
  float* As = smem + grp * 2 * (ASZ + BSZ);
  float* Bs = As + 2 * ASZ;
  const rsrc_t rx = make_rsrc(a.X, (int64_t)a.n * a.ldx);
  const rsrc_t ro = make_rsrc(a.om, (int64_t)a.d * a.R);
  f4 xa[A4], ob[B4];
  auto load = [&](int k0) {
#pragma unroll
    for (int j = 0; j < A4; ++j) {
      const int q = gt + TPG * j, r = q / (BK / 4), k = k0 + 4 * (q % (BK / 4)), row = m0 + r;
      xa[j] = bload4(rx, q < BM * BK / 4 && row < a.n && k < a.d
                             ? (uint32_t)(((int64_t)row * a.ldx + k) * 4) : DGPRF_OOB);
    }
#pragma unroll
    for (int j = 0; j < B4; ++j) {
      const int q = gt + TPG * j, k = k0 + q / (BN / 4), c = n0 + 4 * (q % (BN / 4));
      ob[j] = bload4(ro, q < BN * BK / 4 && k < a.d && c < a.R
                             ? (uint32_t)(((int64_t)k * a.R + c) * 4) : DGPRF_OOB);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < A4; ++j) {
      const int q = gt + TPG * j, r = q / (BK / 4), kq = q % (BK / 4);
      if (q < BM * BK / 4) *reinterpret_cast<f4*>(As + buf * ASZ + (kq * BM + r) * 4) = xa[j];
    }
#pragma unroll
    for (int j = 0; j < B4; ++j) {
      const int q = gt + TPG * j, k = q / (BN / 4), c = 4 * (q % (BN / 4));
      if (q < BN * BK / 4) *reinterpret_cast<f4*>(Bs + buf * BSZ + k * BST + c) = ob[j];
    }
  };
  f4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f4zero();
  const int nkb = (a.d + BK - 1) / BK;
  const int nit = (nkb + KS - 1) / KS;  // iterations; group g runs block it * KS + g
  if (grp < nkb) load(grp * BK);
  store(0);
  __syncthreads();
  for (int it = 0; it < nit; ++it) {
    const int buf = it & 1;
    const int kb_next = (it + 1) * KS + grp;
    if (kb_next < nkb) load(kb_next * BK);
    if (it * KS + grp < nkb) {
      const float* ap = As + buf * ASZ + ((wr * WM + lr) * 4 + lq);
      const float* bp = Bs + buf * BSZ + lq * BST + wc * WN + lr;
      float av[2][MT], bv[2][NT];
#pragma unroll
      for (int i = 0; i < MT; ++i) av[0][i] = ap[16 * i * 4];
#pragma unroll
      for (int j = 0; j < NT; ++j) bv[0][j] = bp[16 * j];
#pragma unroll
      for (int kq = 0; kq < BK / 4; ++kq) {
        const int c = kq & 1;
        if (kq + 1 < BK / 4) {
#pragma unroll
          for (int i = 0; i < MT; ++i) av[c ^ 1][i] = ap[(kq + 1) * BM * 4 + 16 * i * 4];
#pragma unroll
          for (int j = 0; j < NT; ++j) bv[c ^ 1][j] = bp[4 * (kq + 1) * BST + 16 * j];
        }
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NT; ++j) acc[i][j] = mfma16(av[c][i], bv[c][j], acc[i][j]);
      }
    }
    if (it + 1 < nit) store(buf ^ 1);
    __syncthreads();
  }
  // D[i = 4 lq + r][j = lr] of each 16 x 16 tile; k groups summed in group order through LDS
  if (KS > 1) {
    constexpr int PER = MT * NT * 4 * 64;  // floats per wave
    float* red = smem;
    for (int g = KS - 1; g >= 1; --g) {
      if (grp == g) {
        float* p = red + gw * PER + lane;
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) p[((i * NT + j) * 4 + r) * 64] = acc[i][j][r];
      }
      __syncthreads();
      if (grp == g - 1) {
        const float* p = red + gw * PER + lane;
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[i][j][r] += p[((i * NT + j) * 4 + r) * 64];
      }
      __syncthreads();
    }
  }
  if (grp == 0) {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int col = n0 + wc * WN + 16 * j + lr;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + wr * WM + 16 * i + 4 * lq + r;
          if (row < a.n_out && col < a.R) a.out[(int64_t)row * a.R + col] = row < a.n ? acc[i][j][r] : 0.f;
        }
      }
  }
}


// ---------------------------------------------------------------- V3: v1 + two-deep global prefetch
// The load of block kb + 2 is issued at the start of block kb into register stage kb % 2 and
// written to LDS at the end of block kb + 1: two blocks of compute cover its latency.  PERS:
// persistent workgroups (grid = PERS x CUs) looping over tiles.
template <int BM, int BN, int WM, int WN, int PERS>
__global__ __launch_bounds__(256) void k_v3(const Args a, int n_tiles) {
  constexpr int BK = 32;
  constexpr int MT = WM / 32, NT = WN / 32;
  constexpr int AST = BM + 1;
  constexpr int A4 = BM * BK / 4 / 256, B4 = BN * BK / 4 / 256;
  __shared__ float As[2][BK * AST];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK * BN];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wr = wave / (BN / WN), wc = wave % (BN / WN);
  const rsrc_t rx = make_rsrc(a.X, (int64_t)a.n * a.ldx);
  const rsrc_t ro = make_rsrc(a.om, (int64_t)a.d * a.R);
  const int li = lane & 31, lk = lane >> 5;
  const int nkb = (a.d + BK - 1) / BK;
  for (int tile = blockIdx.x; tile < n_tiles; tile += (PERS ? gridDim.x : n_tiles)) {
    const int mt = tile % a.n_mt, ntile = tile / a.n_mt;
    const int m0 = mt * BM, n0 = ntile * BN;
    f4 xa[2][A4], ob[2][B4];
    auto load = [&](int st, int k0) {
#pragma unroll
      for (int j = 0; j < A4; ++j) {
        const int q = tid + 256 * j, r = q / (BK / 4), k = k0 + 4 * (q % (BK / 4)), row = m0 + r;
        xa[st][j] = bload4(rx, row < a.n && k < a.d ? (uint32_t)(((int64_t)row * a.ldx + k) * 4) : DGPRF_OOB);
      }
#pragma unroll
      for (int j = 0; j < B4; ++j) {
        const int q = tid + 256 * j, k = k0 + q / (BN / 4), c = n0 + 4 * (q % (BN / 4));
        ob[st][j] = bload4(ro, k < a.d && c < a.R ? (uint32_t)(((int64_t)k * a.R + c) * 4) : DGPRF_OOB);
      }
    };
    auto store = [&](int st, int buf) {
#pragma unroll
      for (int j = 0; j < A4; ++j) {
        const int q = tid + 256 * j, r = q / (BK / 4), k = 4 * (q % (BK / 4));
#pragma unroll
        for (int c = 0; c < 4; ++c) As[buf][(k + c) * AST + r] = xa[st][j][c];
      }
#pragma unroll
      for (int j = 0; j < B4; ++j) {
        const int q = tid + 256 * j, k = q / (BN / 4), c = 4 * (q % (BN / 4));
        *reinterpret_cast<f4*>(&Bs[buf][k * BN + c]) = ob[st][j];
      }
    };
    f16v acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    auto compute = [&](int buf) {
      const float* ap = &As[buf][lk * AST + wr * WM + li];
      const float* bp = &Bs[buf][lk * BN + wc * WN + li];
#pragma unroll
      for (int ks = 0; ks < BK / 2; ++ks) {
        float av[MT], bv[NT];
#pragma unroll
        for (int i = 0; i < MT; ++i) av[i] = ap[2 * ks * AST + 32 * i];
#pragma unroll
        for (int j = 0; j < NT; ++j) bv[j] = bp[2 * ks * BN + 32 * j];
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NT; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);
      }
    };
    load(0, 0);
    if (nkb > 1) load(1, BK);
    store(0, 0);
    __syncthreads();
    // blocks in pairs so the register stage index stays compile-time
    for (int kb = 0; kb < nkb; kb += 2) {
      if (kb + 2 < nkb) load(0, (kb + 2) * BK);
      compute(0);
      if (kb + 1 < nkb) store(1, 1);
      __syncthreads();
      if (kb + 1 >= nkb) break;
      if (kb + 3 < nkb) load(1, (kb + 3) * BK);
      compute(1);
      if (kb + 2 < nkb) store(0, 0);
      __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int col = n0 + wc * WN + 32 * j + li;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wr * WM + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
          if (row < a.n_out && col < a.R) a.out[(int64_t)row * a.R + col] = row < a.n ? acc[i][j][r] : 0.f;
        }
      }
  }
}

template <int BM, int BN, int WM, int WN, int PERS>
float run_v3(Args a, int reps) {
  a.n_mt = (a.n_out + BM - 1) / BM;
  const int n_tiles = a.n_mt * ((a.R + BN - 1) / BN);
  dim3 grid(PERS ? 256 * PERS : n_tiles);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((k_v3<BM, BN, WM, WN, PERS>), grid, dim3(256), 0, 0, a, n_tiles);
  CK(hipGetLastError());
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((k_v3<BM, BN, WM, WN, PERS>), grid, dim3(256), 0, 0, a, n_tiles);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / reps;
}

template <int BM, int BN, int WM, int WN, int PF, int EPI = 0>
float run_v1(Args a, int reps) {
  a.n_mt = (a.n_out + BM - 1) / BM;
  dim3 grid(a.n_mt * ((a.R + BN - 1) / BN), a.ksplit);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((k_v1<BM, BN, WM, WN, PF, EPI>), grid, dim3(256), 0, 0, a);
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((k_v1<BM, BN, WM, WN, PF, EPI>), grid, dim3(256), 0, 0, a);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / reps;
}

template <int BM, int BN, int WM, int WN, int KS, int BK>
float run_v2(Args a, int reps) {
  constexpr int NT = 64 * (BM / WM) * (BN / WN) * KS;
  const size_t lds = (size_t)KS * 2 * (BK * BM + BK * (BN + 16)) * 4;
  const size_t red = (size_t)(BM / WM) * (BN / WN) * (WM / 16) * (WN / 16) * 4 * 64 * 4;
  const size_t L = lds > red ? lds : red;
  if (L > 160 * 1024) return -1.f;
  CK(hipFuncSetAttribute((const void*)k_v2<BM, BN, WM, WN, KS, BK>,
                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)L));
  a.n_mt = (a.n_out + BM - 1) / BM;
  dim3 grid(a.n_mt * ((a.R + BN - 1) / BN));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((k_v2<BM, BN, WM, WN, KS, BK>), grid, dim3(NT), L, 0, a);
  CK(hipGetLastError());
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((k_v2<BM, BN, WM, WN, KS, BK>), grid, dim3(NT), L, 0, a);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / reps;
}

// ---------------------------------------------------------------- V5: v1 with split K over SK
// workgroups (blockIdx.y = K part; part p writes its own [n_out][R] slab, summed by the consumer):
// SK x the workgroups, so two or more of them share a CU and one computes while another waits on
// its block loads (the in-workgroup K split of v2 shares one barrier per block and does not).
template <int BM, int BN, int WM, int WN, int SK>
__global__ __launch_bounds__(256) void k_v5(const Args a) {
  constexpr int BK = 32;
  constexpr int MT = WM / 32, NT = WN / 32;
  constexpr int AST = BM + 1;
  constexpr int A4 = BM * BK / 4 / 256, B4 = BN * BK / 4 / 256;
  __shared__ float As[2][BK * AST];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK * BN];
  int mt, ntile;
  tile_of(a, blockIdx.x, gridDim.x, mt, ntile);
  const int m0 = mt * BM, n0 = ntile * BN;
  const int part = blockIdx.y;
  // K range of this part, whole k-blocks: [kb0, kb1) of the d / BK blocks
  const int nkb_all = (a.d + BK - 1) / BK;
  const int kb0 = nkb_all * part / SK, kb1 = nkb_all * (part + 1) / SK;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wr = wave / (BN / WN), wc = wave % (BN / WN);
  const rsrc_t rx = make_rsrc(a.X, (int64_t)a.n * a.ldx);
  const rsrc_t ro = make_rsrc(a.om, (int64_t)a.d * a.R);
  f4 xa[A4], ob[B4];
  auto load = [&](int k0) {
#pragma unroll
    for (int j = 0; j < A4; ++j) {
      const int q = tid + 256 * j, r = q / (BK / 4), k = k0 + 4 * (q % (BK / 4)), row = m0 + r;
      xa[j] = bload4(rx, row < a.n && k < a.d ? (uint32_t)(((int64_t)row * a.ldx + k) * 4) : DGPRF_OOB);
    }
#pragma unroll
    for (int j = 0; j < B4; ++j) {
      const int q = tid + 256 * j, k = k0 + q / (BN / 4), c = n0 + 4 * (q % (BN / 4));
      ob[j] = bload4(ro, k < a.d && c < a.R ? (uint32_t)(((int64_t)k * a.R + c) * 4) : DGPRF_OOB);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < A4; ++j) {
      const int q = tid + 256 * j, r = q / (BK / 4), k = 4 * (q % (BK / 4));
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
  load(kb0 * BK);
  store(0);
  __syncthreads();
  const int li = lane & 31, lk = lane >> 5;
  for (int kb = kb0; kb < kb1; ++kb) {
    const int buf = (kb - kb0) & 1;
    if (kb + 1 < kb1) load((kb + 1) * BK);
    const float* ap = &As[buf][lk * AST + wr * WM + li];
    const float* bp = &Bs[buf][lk * BN + wc * WN + li];
#pragma unroll
    for (int ks = 0; ks < BK / 2; ++ks) {
      float av[MT], bv[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i) av[i] = ap[2 * ks * AST + 32 * i];
#pragma unroll
      for (int j = 0; j < NT; ++j) bv[j] = bp[2 * ks * BN + 32 * j];
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    if (kb + 1 < kb1) store(buf ^ 1);
    __syncthreads();
  }
  float* out = a.out + (int64_t)part * a.n_out * a.R;
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int col = n0 + wc * WN + 32 * j + li;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wr * WM + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (row < a.n_out && col < a.R) out[(int64_t)row * a.R + col] = row < a.n ? acc[i][j][r] : 0.f;
      }
    }
}

template <int BM, int BN, int WM, int WN, int SK>
float run_v5(Args a, int reps) {
  a.n_mt = (a.n_out + BM - 1) / BM;
  dim3 grid(a.n_mt * ((a.R + BN - 1) / BN), SK);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((k_v5<BM, BN, WM, WN, SK>), grid, dim3(256), 0, 0, a);
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((k_v5<BM, BN, WM, WN, SK>), grid, dim3(256), 0, 0, a);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / reps;
}

// ---------------------------------------------------------------- V6: deep prefetch
// v1's compute, with the Omega blocks copied global -> LDS by buffer_load ... lds (no VGPRs, OOB
// rows read as 0) into a 4-slot ring three blocks ahead, and the X blocks loaded three blocks ahead
// into a 3-slot register ring (static slots: the block loop is unrolled by 3), transposed into a
// double-buffered LDS image one block ahead.  One barrier per block; vmcnt counts the younger
// blocks' loads that may stay in flight.
template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(256) void k_v6(const Args a) {
  constexpr int BK = 32, NS = 4;
  constexpr int MT = WM / 32, NT = WN / 32;
  constexpr int AST = BM + 1;
  constexpr int A4 = BM * BK / 4 / 256;
  constexpr int OPW = BK * BN / 256 / 4;  // 1-KiB LDS-DMA pieces per wave per block
  constexpr int PER = A4 + OPW;           // vector-memory instructions per wave per block
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* As = sm;                 // [2][BK * AST]
  float* Bs = sm + 2 * BK * AST;  // [NS][BK * BN]
  int mt, ntile;
  tile_of(a, blockIdx.x, gridDim.x, mt, ntile);
  const int m0 = mt * BM, n0 = ntile * BN;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wr = wave / (BN / WN), wc = wave % (BN / WN);
  const rsrc_t rx = make_rsrc(a.X, (int64_t)a.n * a.ldx);
  const rsrc_t ro = make_rsrc(a.om, (int64_t)a.d * a.R);
  const int nkb = (a.d + BK - 1) / BK;
  f4 x0[A4], x1[A4], x2[A4];
  auto xload = [&](int kb, f4 (&x)[A4]) {
#pragma unroll
    for (int j = 0; j < A4; ++j) {
      const int q = tid + 256 * j, r = q / (BK / 4), k = kb * BK + 4 * (q % (BK / 4)), row = m0 + r;
      x[j] = bload4(rx, row < a.n && k < a.d ? (uint32_t)(((int64_t)row * a.ldx + k) * 4) : DGPRF_OOB);
    }
  };
  auto xstore = [&](int kb, const f4 (&x)[A4]) {
    float* dst = As + (kb & 1) * BK * AST;
#pragma unroll
    for (int j = 0; j < A4; ++j) {
      const int q = tid + 256 * j, r = q / (BK / 4), k = 4 * (q % (BK / 4));
#pragma unroll
      for (int c = 0; c < 4; ++c) dst[(k + c) * AST + r] = x[j][c];
    }
  };
  auto odma = [&](int kb) {
    float* dst = Bs + (kb % NS) * BK * BN;
#pragma unroll
    for (int j = 0; j < OPW; ++j) {
      const int piece = wave * OPW + j, e = piece * 256 + lane * 4;
      const int row = e / BN, col = e % BN, k = kb * BK + row, c = n0 + col;
      const uint32_t off = k < a.d && c < a.R ? (uint32_t)(((int64_t)k * a.R + c) * 4) : DGPRF_OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ro, (__attribute__((address_space(3))) void*)(dst + piece * 256),
                                               16, off, 0, 0, 0);
    }
  };
  f16v acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int li = lane & 31, lk = lane >> 5;
  auto compute = [&](int kb) {
    const float* ap = As + (kb & 1) * BK * AST + lk * AST + wr * WM + li;
    const float* bp = Bs + (kb % NS) * BK * BN + lk * BN + wc * WN + li;
#pragma unroll
    for (int ks = 0; ks < BK / 2; ++ks) {
      float av[MT], bv[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i) av[i] = ap[2 * ks * AST + 32 * i];
#pragma unroll
      for (int j = 0; j < NT; ++j) bv[j] = bp[2 * ks * BN + 32 * j];
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
  };
  // prologue: blocks 0..2 in flight, block 0 landed
  xload(0, x0); odma(0);
  if (1 < nkb) { xload(1, x1); odma(1); }
  if (2 < nkb) { xload(2, x2); odma(2); }
  if (2 < nkb) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * PER) : "memory");
  else if (1 < nkb) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(PER) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  xstore(0, x0);
  // raw barrier: __syncthreads() adds a fence whose wait drains every load in flight (vmcnt(0)),
  // which would end the prefetch; the X image's LDS writes are waited for explicitly instead
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  // block kb: issue block kb + 3 into the slot block kb freed, compute kb, land and stage kb + 1
  auto body = [&](int kb, f4 (&xs_new)[A4], const f4 (&xs_next)[A4]) {
    if (kb + 3 < nkb) { xload(kb + 3, xs_new); odma(kb + 3); }
    compute(kb);
    if (kb + 1 < nkb) {
      if (kb + 3 < nkb) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * PER) : "memory");
      else if (kb + 2 < nkb) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(PER) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      xstore(kb + 1, xs_next);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  for (int kb = 0; kb < nkb; kb += 3) {
    body(kb, x0, x1);
    if (kb + 1 < nkb) body(kb + 1, x1, x2);
    if (kb + 2 < nkb) body(kb + 2, x2, x0);
  }
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int col = n0 + wc * WN + 32 * j + li;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wr * WM + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (row < a.n_out && col < a.R) a.out[(int64_t)row * a.R + col] = row < a.n ? acc[i][j][r] : 0.f;
      }
    }
}

template <int BM, int BN, int WM, int WN>
float run_v6(Args a, int reps) {
  const size_t L = (size_t)(2 * 32 * (BM + 1) + 4 * 32 * BN) * 4;
  CK(hipFuncSetAttribute((const void*)k_v6<BM, BN, WM, WN>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)L));
  a.n_mt = (a.n_out + BM - 1) / BM;
  dim3 grid(a.n_mt * ((a.R + BN - 1) / BN));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((k_v6<BM, BN, WM, WN>), grid, dim3(256), L, 0, a);
  CK(hipGetLastError());
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((k_v6<BM, BN, WM, WN>), grid, dim3(256), L, 0, a);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / reps;
}

// ---------------------------------------------------------------- V7: every block by LDS-DMA
// X and Omega blocks copied global -> LDS by buffer_load ... lds (no registers, nothing for the
// compiler's wait counting to serialise) into 4-slot rings, issued three blocks ahead; X is
// transposed LDS -> LDS into a 3-slot k-major image two blocks ahead, right after the one barrier
// per block (which also covers the DMA of that block: every wave waits for its own pieces first).
template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(256) void k_v7(const Args a) {
  constexpr int BK = 32, NS = 4;
  constexpr int MT = WM / 32, NT = WN / 32;
  constexpr int AST = BM + 1;
  constexpr int XPW = BM * BK / 256 / 4;  // 1-KiB X pieces per wave per block
  constexpr int OPW = BK * BN / 256 / 4;  // 1-KiB Omega pieces per wave per block
  constexpr int PER = XPW + OPW;
  static_assert(XPW >= 1 && OPW >= 1, "tile too small");
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* Bs = sm;                          // [NS][BK * BN]
  float* Xs = Bs + NS * BK * BN;           // [NS][BM * BK] row-major staging
  float* As = Xs + NS * BM * BK;           // [3][BK * AST] k-major
  int mt, ntile;
  tile_of(a, blockIdx.x, gridDim.x, mt, ntile);
  const int m0 = mt * BM, n0 = ntile * BN;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wr = wave / (BN / WN), wc = wave % (BN / WN);
  const rsrc_t rx = make_rsrc(a.X, (int64_t)a.n * a.ldx);
  const rsrc_t ro = make_rsrc(a.om, (int64_t)a.d * a.R);
  const int nkb = (a.d + BK - 1) / BK;
  auto issue = [&](int kb) {
    float* xd = Xs + (kb % NS) * BM * BK;
#pragma unroll
    for (int j = 0; j < XPW; ++j) {
      const int piece = wave * XPW + j, e = piece * 256 + lane * 4;
      const int row = e / BK, k = kb * BK + e % BK, r = m0 + row;
      const uint32_t off = r < a.n && k < a.d ? (uint32_t)(((int64_t)r * a.ldx + k) * 4) : DGPRF_OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (__attribute__((address_space(3))) void*)(xd + piece * 256),
                                               16, off, 0, 0, 0);
    }
    float* od = Bs + (kb % NS) * BK * BN;
#pragma unroll
    for (int j = 0; j < OPW; ++j) {
      const int piece = wave * OPW + j, e = piece * 256 + lane * 4;
      const int row = e / BN, col = e % BN, k = kb * BK + row, c = n0 + col;
      const uint32_t off = k < a.d && c < a.R ? (uint32_t)(((int64_t)k * a.R + c) * 4) : DGPRF_OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ro, (__attribute__((address_space(3))) void*)(od + piece * 256),
                                               16, off, 0, 0, 0);
    }
  };
  auto transpose = [&](int kb) {  // staging slot kb % NS -> k-major image kb % 3
    const float* xs = Xs + (kb % NS) * BM * BK;
    float* ad = As + (kb % 3) * BK * AST;
#pragma unroll
    for (int j = 0; j < BM * BK / 4 / 256; ++j) {
      const int q = tid + 256 * j, r = q / (BK / 4), k = 4 * (q % (BK / 4));
      const f4 v = *reinterpret_cast<const f4*>(xs + r * BK + k);
#pragma unroll
      for (int c = 0; c < 4; ++c) ad[(k + c) * AST + r] = v[c];
    }
  };
  f16v acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int li = lane & 31, lk = lane >> 5;
  auto compute = [&](int kb) {
    const float* ap = As + (kb % 3) * BK * AST + lk * AST + wr * WM + li;
    const float* bp = Bs + (kb % NS) * BK * BN + lk * BN + wc * WN + li;
#pragma unroll
    for (int ks = 0; ks < BK / 2; ++ks) {
      float av[MT], bv[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i) av[i] = ap[2 * ks * AST + 32 * i];
#pragma unroll
      for (int j = 0; j < NT; ++j) bv[j] = bp[2 * ks * BN + 32 * j];
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
  };
  auto sync = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  // prologue: blocks 0..2 issued; 0 and 1 landed and transposed
  issue(0);
  if (1 < nkb) issue(1);
  if (2 < nkb) issue(2);
  if (2 < nkb) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(PER) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  sync();
  transpose(0);
  if (1 < nkb) transpose(1);
  sync();
  for (int kb = 0; kb < nkb; ++kb) {
    if (kb + 3 < nkb) issue(kb + 3);
    compute(kb);
    if (kb + 2 < nkb) {  // block kb + 2 landed (only kb + 3 may be in flight), then transposed
      if (kb + 3 < nkb) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(PER) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      sync();
      transpose(kb + 2);
    }
    sync();  // (two barriers only when a transpose ran: its image is read two blocks later)
  }
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int col = n0 + wc * WN + 32 * j + li;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wr * WM + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (row < a.n_out && col < a.R) a.out[(int64_t)row * a.R + col] = row < a.n ? acc[i][j][r] : 0.f;
      }
    }
}

template <int BM, int BN, int WM, int WN>
float run_v7(Args a, int reps) {
  const size_t L = (size_t)(4 * 32 * BN + 4 * BM * 32 + 3 * 32 * (BM + 1)) * 4;
  if (L > 160 * 1024) return -1.f;
  CK(hipFuncSetAttribute((const void*)k_v7<BM, BN, WM, WN>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)L));
  a.n_mt = (a.n_out + BM - 1) / BM;
  dim3 grid(a.n_mt * ((a.R + BN - 1) / BN));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((k_v7<BM, BN, WM, WN>), grid, dim3(256), L, 0, a);
  CK(hipGetLastError());
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((k_v7<BM, BN, WM, WN>), grid, dim3(256), L, 0, a);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / reps;
}

// ---------------------------------------------------------------- V8: v1 with k-split wave groups
// KS groups of (BM/WM)*(BN/WN) waves; group g runs k-blocks g, g + KS, ... with its own double
// buffer (register-staged like v1), one barrier per KS blocks; the group accumulators are summed
// in LDS at the end (group order).  BK: k-block depth.
template <int BM, int BN, int WM, int WN, int KS, int BK>
__global__ __launch_bounds__(64 * (BM / WM) * (BN / WN) * KS) void k_v8(const Args a) {
  constexpr int WPG = (BM / WM) * (BN / WN), TPG = 64 * WPG;
  constexpr int MT = WM / 32, NT = WN / 32;
  constexpr int AST = BM + 1;
  constexpr int A4 = BM * BK / 4 / TPG, B4 = BN * BK / 4 / TPG;
  static_assert(A4 >= 1 && B4 >= 1 && BM * BK / 4 % TPG == 0 && BN * BK / 4 % TPG == 0, "tile");
  constexpr int GSZ = 2 * BK * (AST + BN);  // floats per group
  extern __shared__ __attribute__((aligned(16))) float sm[];
  int mt, ntile;
  tile_of(a, blockIdx.x, gridDim.x, mt, ntile);
  const int m0 = mt * BM, n0 = ntile * BN;
  const int tid = threadIdx.x, grp = tid / TPG, gt = tid % TPG;
  const int wave = gt >> 6, lane = tid & 63;
  const int wr = wave / (BN / WN), wc = wave % (BN / WN);
  float* As = sm + grp * GSZ;            // [2][BK * AST]
  float* Bs = As + 2 * BK * AST;         // [2][BK * BN]
  const rsrc_t rx = make_rsrc(a.X, (int64_t)a.n * a.ldx);
  const rsrc_t ro = make_rsrc(a.om, (int64_t)a.d * a.R);
  f4 xa[A4], ob[B4];
  auto load = [&](int k0) {
#pragma unroll
    for (int j = 0; j < A4; ++j) {
      const int q = gt + TPG * j, r = q / (BK / 4), k = k0 + 4 * (q % (BK / 4)), row = m0 + r;
      xa[j] = bload4(rx, row < a.n && k < a.d ? (uint32_t)(((int64_t)row * a.ldx + k) * 4) : DGPRF_OOB);
    }
#pragma unroll
    for (int j = 0; j < B4; ++j) {
      const int q = gt + TPG * j, k = k0 + q / (BN / 4), c = n0 + 4 * (q % (BN / 4));
      ob[j] = bload4(ro, k < a.d && c < a.R ? (uint32_t)(((int64_t)k * a.R + c) * 4) : DGPRF_OOB);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < A4; ++j) {
      const int q = gt + TPG * j, r = q / (BK / 4), k = 4 * (q % (BK / 4));
#pragma unroll
      for (int c = 0; c < 4; ++c) As[buf * BK * AST + (k + c) * AST + r] = xa[j][c];
    }
#pragma unroll
    for (int j = 0; j < B4; ++j) {
      const int q = gt + TPG * j, k = q / (BN / 4), c = 4 * (q % (BN / 4));
      *reinterpret_cast<f4*>(&Bs[buf * BK * BN + k * BN + c]) = ob[j];
    }
  };
  f16v acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int nkb = (a.d + BK - 1) / BK;
  const int nit = (nkb + KS - 1) / KS;  // iterations; group g's block of iteration i: i * KS + g
  load(grp * BK);                       // (k beyond d stages zeros)
  store(0);
  __syncthreads();
  const int li = lane & 31, lk = lane >> 5;
  for (int it = 0; it < nit; ++it) {
    const int buf = it & 1;
    if (it + 1 < nit) load(((it + 1) * KS + grp) * BK);
    const float* ap = As + buf * BK * AST + lk * AST + wr * WM + li;
    const float* bp = Bs + buf * BK * BN + lk * BN + wc * WN + li;
#pragma unroll
    for (int ks = 0; ks < BK / 2; ++ks) {
      float av[MT], bv[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i) av[i] = ap[2 * ks * AST + 32 * i];
#pragma unroll
      for (int j = 0; j < NT; ++j) bv[j] = bp[2 * ks * BN + 32 * j];
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    if (it + 1 < nit) store(buf ^ 1);
    __syncthreads();
  }
  if (KS > 1) {  // groups 1.. add theirs into group 0's in order (per-wave 32x32 blocks via LDS)
    float* red = sm + (size_t)wave * (MT * NT * 1024);
#pragma unroll
    for (int g = 1; g < KS; ++g) {
      if (grp == g)
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) red[((i * NT + j) * 16 + r) * 64 + lane] = acc[i][j][r];
      __syncthreads();
      if (grp == 0)
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] += red[((i * NT + j) * 16 + r) * 64 + lane];
      __syncthreads();
    }
    if (grp != 0) return;
  }
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int col = n0 + wc * WN + 32 * j + li;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wr * WM + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (row < a.n_out && col < a.R) a.out[(int64_t)row * a.R + col] = row < a.n ? acc[i][j][r] : 0.f;
      }
    }
}

template <int BM, int BN, int WM, int WN, int KS, int BK>
float run_v8(Args a, int reps) {
  constexpr int WPG = (BM / WM) * (BN / WN);
  const size_t L = (size_t)KS * 2 * BK * (BM + 1 + BN) * 4;
  if (L > 160 * 1024) return -1.f;
  auto fn = k_v8<BM, BN, WM, WN, KS, BK>;
  CK(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)L));
  a.n_mt = (a.n_out + BM - 1) / BM;
  dim3 grid(a.n_mt * ((a.R + BN - 1) / BN));
  const dim3 blk(64 * WPG * KS);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(fn, grid, blk, L, 0, a);
  CK(hipGetLastError());
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(fn, grid, blk, L, 0, a);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / reps;
}

static double check(const std::vector<float>& hx, const std::vector<float>& ho, const float* dout,
                    int n, int n_out, int d, int R, int parts = 1) {
  std::vector<float> out((size_t)n_out * R), tmp((size_t)n_out * R);
  CK(hipMemcpy(out.data(), dout, out.size() * 4, hipMemcpyDeviceToHost));
  for (int p = 1; p < parts; ++p) {
    CK(hipMemcpy(tmp.data(), dout + (size_t)p * n_out * R, tmp.size() * 4, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < out.size(); ++i) out[i] += tmp[i];
  }
  std::mt19937 g(5);
  double worst = 0;
  for (int t = 0; t < 2000; ++t) {
    const int i = g() % n_out, j = g() % R;
    double ref = 0, sc = 0;
    if (i < n)
      for (int k = 0; k < d; ++k) {
        ref += (double)hx[(size_t)i * d + k] * ho[(size_t)k * R + j];
        sc += std::fabs((double)hx[(size_t)i * d + k] * ho[(size_t)k * R + j]);
      }
    const double e = std::fabs(out[(size_t)i * R + j] - ref) / (sc + 1e-30);
    worst = e > worst ? e : worst;
  }
  CK(hipMemset((void*)dout, 0xff, out.size() * 4));
  return worst;
}

int main() {
  const int d = 784, R = 4096, nmax = 10000;
  std::vector<float> hx((size_t)nmax * d), ho((size_t)d * R);
  std::mt19937 g(1);
  std::uniform_real_distribution<float> u(-1.f, 1.f);
  for (auto& v : hx) v = u(g);
  for (auto& v : ho) v = u(g);
  float *X, *O, *Y;
  CK(hipMalloc(&X, hx.size() * 4));
  CK(hipMalloc(&O, ho.size() * 4));
  CK(hipMalloc(&Y, (size_t)4 * nmax * R * 4));
  CK(hipMemcpy(X, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(O, ho.data(), ho.size() * 4, hipMemcpyHostToDevice));
  struct Shape {
    const char* name;
    int n, n_out, reps;
  } shapes[] = {{"step 200(224)x784x4096", 200, 224, 200}, {"pred 10000x784x4096", 10000, 10000, 20}};
  for (const Shape& s : shapes) {
    Args a{X, O, Y, s.n, s.n_out, d, d, R, 0, 0, 1};
    const double fl = 2.0 * s.n * (double)d * R;
    auto rep = [&](const char* v, float us, int parts = 1) {
      if (us < 0) {
        printf("%-24s %-34s (LDS too large)\n", s.name, v);
        return;
      }
      const double err = check(hx, ho, Y, s.n, s.n_out, d, R, parts);
      printf("%-24s %-34s %9.2f us  %6.1f TF  err %.2e\n", s.name, v, us, fl / (us * 1e-6) / 1e12, err);
      fflush(stdout);
    };
    if (s.n_out <= 1024) {
      a.gm = 1000;
      a.ksplit = 2;
      rep("v1 64x64 w32x32 pf3 xcd sk2", run_v1<64, 64, 32, 32, 3>(a, s.reps), 2);
      rep("v1 64x64 w32x32 pf3 xcd sk2 epi", run_v1<64, 64, 32, 32, 3, 1>(a, s.reps), 2);
      a.ksplit = 1;
      a.gm = 0;
    } else {
      rep("v1 128x128 w64x64 pf0", run_v1<128, 128, 64, 64, 0>(a, s.reps));
      rep("v1 64x64 w32x32 pf0", run_v1<64, 64, 32, 32, 0>(a, s.reps));
      rep("v1 64x64 w32x32 pf3", run_v1<64, 64, 32, 32, 3>(a, s.reps));
      a.gm = 8;
      rep("v1 64x64 w32x32 pf3 xcd gm8", run_v1<64, 64, 32, 32, 3>(a, s.reps));
      a.gm = 0;
      rep("v1 64x128 w32x64 pf3", run_v1<64, 128, 32, 64, 3>(a, s.reps));
      rep("v1 128x64 w64x32 pf3", run_v1<128, 64, 64, 32, 3>(a, s.reps));
      rep("v1 128x128 w64x64 pf0 (again)", run_v1<128, 128, 64, 64, 0>(a, s.reps));
    }
  }
  return 0;
}
