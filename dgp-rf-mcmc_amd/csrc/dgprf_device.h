// dgprf_device.h — device helpers shared by the gfx950 kernels of libdgprf.so.
//
//  * MFMA: v_mfma_f32_16x16x4_f32 (exact fp32 fma chain).  Lane maps (CDNA4, wave64):
//      A[i = lane&15][k = lane>>4],  B[k = lane>>4][j = lane&15],
//      D[i = 4*(lane>>4) + reg][j = lane&15]          (reg = 0..3)
//  * Philox4x32-10 counter RNG + Box-Muller: the device replacement of TF's stateful
//    tf.random.normal (layers/rf_layers.py:22, layers/GP_weight_layers.py:9, models/dgp.py:210-212).
//  * keyed Feistel permutation: the on-device replacement of tf.data's per-epoch shuffle +
//    drop-remainder batching (experiments/utils_dataset.py:38-42).
// The oracle (oracle/rng.py) restates Philox and Feistel bit-exactly for the tests.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dgprf.h"

typedef float f4 __attribute__((ext_vector_type(4)));

#define DGPRF_WAVES 4
#define DGPRF_TILE_ROWS 16
#define DGPRF_NS_MAX 16  // feature slices per step kernel (partial buffers are padded to it)

__device__ __forceinline__ f4 mfma16(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// v_mfma_f32_4x4x1_16b_f32: 16 independent 4x4x1 blocks, block b = lanes 4b..4b+3 (measured,
// scripts/microbench/mfma4x4.hip):  A_b[i] = lane 4b+i,  B_b[j] = lane 4b+j,  D_b[i][j] = lane 4b+j
// reg i.  256 MACs per ~8-12 cycles: the fit for contractions whose output width is <= 8.
__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f4 f4zero() {
  f4 z = {0.f, 0.f, 0.f, 0.f};
  return z;
}

// ---------------------------------------------------------------- buffer loads
// Raw buffer loads through a wave-uniform descriptor: lanes with an offset past the descriptor's
// size (OOB) read 0 without a memory access, so masked lanes cost no traffic and every load of a
// burst can be unconditional.
constexpr uint32_t DGPRF_OOB = 0x80000000u;
typedef __amdgpu_buffer_rsrc_t rsrc_t;

__device__ __forceinline__ rsrc_t make_rsrc(const float* p, int64_t n_floats) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)(n_floats * 4), 0x00020000);
}
// The same, for call sites whose pointer / size the compiler cannot prove wave-uniform (values
// derived through selects or dynamically indexed kernel-argument arrays): both go through
// readfirstlane, so the descriptor is built in SGPRs instead of a waterfall loop around every load.
// Only for values that ARE wave-uniform.
__device__ __forceinline__ rsrc_t make_rsrc_u(const float* p, int n_floats) {
  const uint64_t a = (uint64_t)p;
  const uint64_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  const uint64_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(lo | (hi << 32)), (short)0,
                                           __builtin_amdgcn_readfirstlane(n_floats * 4), 0x00020000);
}
__device__ __forceinline__ f4 bload4(rsrc_t r, uint32_t byte_off) {
  return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0));
}
__device__ __forceinline__ float bload1(rsrc_t r, uint32_t byte_off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, 0));
}
// Write-through store (cache policy sc1): the line goes on to the memory side instead of staying
// dirty in this XCD's L2, so the kernel boundary does not pay its write-back (MI355X_MICROARCH.md,
// price table row 'boundary': + bytes / 6 TB/s behind dirty fp32 partials).
__device__ __forceinline__ void bstore1_wt(float v, rsrc_t r, uint32_t byte_off) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, byte_off, 0, 16);
}
typedef unsigned int u32v4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void bstore4_wt(f4 v, rsrc_t r, uint32_t byte_off) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32v4, v), r, byte_off, 0, 16);
}

// ---------------------------------------------------------------- Philox4x32-10
struct u32x4 {
  uint32_t x, y, z, w;
};

__host__ __device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * (uint64_t)c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * (uint64_t)c.z;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    u32x4 n;
    n.x = hi1 ^ c.y ^ k0;
    n.y = lo1;
    n.z = hi0 ^ c.w ^ k1;
    n.w = lo0;
    c = n;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// Two N(0,1) from two uint32 (Box-Muller, u1 in (0,1], u2 in [0,1), 24-bit grids).
__device__ __forceinline__ void box_muller(uint32_t a, uint32_t b, float* z0, float* z1) {
  const float u1 = (float)((a >> 8) + 1u) * 5.9604644775390625e-08f;  // 2^-24
  const float u2 = (float)(b >> 8) * 5.9604644775390625e-08f;
  const float r = sqrtf(-2.0f * logf(u1));
  float s, c;
  sincospif(2.0f * u2, &s, &c);
  *z0 = r * c;
  *z1 = r * s;
}

// Four normals for counter quad `q` of stream (seed, sub, purpose, lane_tag).
__device__ __forceinline__ f4 philox_normal4(uint64_t seed, uint64_t sub, uint32_t purpose,
                                             uint32_t tag, uint32_t q) {
  u32x4 c;
  c.x = q;
  c.y = (uint32_t)sub;
  c.z = (uint32_t)(sub >> 32);
  c.w = (purpose << 24) | (tag & 0x00FFFFFFu);
  const u32x4 r = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  f4 z;
  float a, b, e, f;
  box_muller(r.x, r.y, &a, &b);
  box_muller(r.z, r.w, &e, &f);
  z[0] = a;
  z[1] = b;
  z[2] = e;
  z[3] = f;
  return z;
}

// ---------------------------------------------------------------- Feistel permutation
__host__ __device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

__host__ __device__ __forceinline__ uint32_t feistel_key(uint64_t seed, uint32_t chain,
                                                         uint64_t epoch, uint32_t round) {
  const uint32_t mix = (uint32_t)(seed >> 32) + chain * 0x632BE5ABu + (uint32_t)epoch * 0x9E3779B9u +
                       (uint32_t)(epoch >> 32) * 0x85EBCA6Bu + round * 0x27D4EB2Fu;
  return fmix32((uint32_t)seed ^ fmix32(mix));
}

// Bijection of [0, n) (n <= 2^32): 4-round balanced Feistel on ceil-even-log2(n) bits with
// cycle walking.
__host__ __device__ __forceinline__ uint32_t feistel_perm(uint32_t x, uint64_t n, uint64_t seed,
                                                          uint32_t chain, uint64_t epoch) {
  uint32_t bits = 2;
  while (bits < 32 && ((uint64_t)1 << bits) < n) bits += 2;
  const uint32_t half = bits >> 1;
  const uint32_t mask = (half >= 32) ? 0xFFFFFFFFu : ((1u << half) - 1u);
  const uint32_t k0 = feistel_key(seed, chain, epoch, 0);
  const uint32_t k1 = feistel_key(seed, chain, epoch, 1);
  const uint32_t k2 = feistel_key(seed, chain, epoch, 2);
  const uint32_t k3 = feistel_key(seed, chain, epoch, 3);
  do {
    uint32_t L = x >> half, R = x & mask;
    uint32_t t;
    t = L ^ (fmix32(R * 0x9E3779B1u + k0) & mask); L = R; R = t;
    t = L ^ (fmix32(R * 0x9E3779B1u + k1) & mask); L = R; R = t;
    t = L ^ (fmix32(R * 0x9E3779B1u + k2) & mask); L = R; R = t;
    t = L ^ (fmix32(R * 0x9E3779B1u + k3) & mask); L = R; R = t;
    x = (L << half) | R;
  } while ((uint64_t)x >= n);
  return x;
}

// ---------------------------------------------------------------- trig
#ifdef DGPRF_PRECISE_TRIG
#define DGPRF_PRECISE_TRIG_ON true
#else
#define DGPRF_PRECISE_TRIG_ON false
#endif
// cos/sin of the RF inner products.  Range-reduce in revolutions (x/2pi - rint) and use the
// hardware v_sin/v_cos (which take revolutions).  DGPRF_PRECISE_TRIG selects ocml sincosf.
__device__ __forceinline__ void rf_sincos(float x, float* s, float* c) {
#ifdef DGPRF_PRECISE_TRIG
  sincosf(x, s, c);
#else
  float t = x * 0.15915494309189535f;
  t = t - rintf(t);
  *s = __builtin_amdgcn_sinf(t);
  *c = __builtin_amdgcn_cosf(t);
#endif
}

// ---------------------------------------------------------------- minibatch rows
struct BatchDev {
  const float* X;
  const float* Y;
  const int32_t* idx;
  int64_t n_data;
  int64_t iters;
  uint64_t perm_seed;
  int32_t y_cols;
  int32_t mode;
  const float* A1;  // resident X Omega_1 [n_data][a1_ld] (wide first layer, fixed Omega_1) or null
  int32_t a1_ld, pad;
};

__device__ __forceinline__ int64_t batch_row(const BatchDev& bd, int B, int chain, int64_t t,
                                             int b) {
  if (bd.mode == DGPRF_BATCH_DIRECT) return b;
  if (bd.mode == DGPRF_BATCH_INDEXED) return bd.idx[(int64_t)chain * B + b];
  const int64_t it = bd.iters > 0 ? bd.iters : 1;
  const int64_t epoch = t / it;
  const int64_t pos = (t % it) * (int64_t)B + b;
  return (int64_t)feistel_perm((uint32_t)pos, (uint64_t)bd.n_data, bd.perm_seed, (uint32_t)chain,
                               (uint64_t)epoch);
}
