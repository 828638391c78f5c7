// mfma_lat.hip — cycle cost of the instruction patterns of the step kernels' compute section
// (one wave per SIMD, s_memtime around each pattern, median over 256 workgroups):
//   A: 8 independent v_mfma_f32_16x16x4_f32 (two accumulators, interleaved)
//   B: 8 dependent MFMAs (one accumulator)
//   C: the feature pattern: 2-MFMA A-tile -> read accumulators -> 4x (rint, fma, sin, cos)
//      -> 8 MFMAs into two accumulators
//   D: like C but the 8 trailing MFMAs replaced by VALU fmas
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
#define MF(a, b, c) __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0)

constexpr int G_ = 256;
__global__ __launch_bounds__(256) void k(const float* in, float* out, unsigned long long* t) {
  const int lane = threadIdx.x & 63;
  float x = in[threadIdx.x], y = in[threadIdx.x + 256];
  const f4 z4 = {0, 0, 0, 0};
  f4 a = z4, b = z4;
  unsigned long long t0, t1, t2, t3, t4;
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_sched_barrier(0);
  t0 = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a = MF(x, y, a);
    b = MF(y, x, b);
  }
  __builtin_amdgcn_sched_barrier(0);
  float s0 = a[0] + b[3];
  t1 = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < 8; ++i) a = MF(x + s0, y, a);
  float s1 = a[1];
  __builtin_amdgcn_sched_barrier(0);
  t2 = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
  {
    f4 at = MF(x, s1, z4);
    at = MF(y, s1, at);
    f4 c = {0, 0, 0, 0}, s = {0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float u = at[r] * 0.15915494f;
      u = u - rintf(u);
      const float cv = __builtin_amdgcn_cosf(u) * 1.1f, sv = __builtin_amdgcn_sinf(u) * 1.1f;
      c = MF(x, cv, c);
      s = MF(y, sv, s);
    }
    s1 = c[0] + s[2];
  }
  __builtin_amdgcn_sched_barrier(0);
  t3 = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
  {
    f4 at = MF(x, s1, z4);
    at = MF(y, s1, at);
    float c = 0.f, s = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float u = at[r] * 0.15915494f;
      u = u - rintf(u);
      c = fmaf(x, __builtin_amdgcn_cosf(u), c);
      s = fmaf(y, __builtin_amdgcn_sinf(u), s);
    }
    s1 += c + s;
  }
  __builtin_amdgcn_sched_barrier(0);
  t4 = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
  {  // E: C with all transcendentals batched before the 8 MFMAs
    f4 at = MF(x, s1, z4);
    at = MF(y, s1, at);
    float cv[4], sv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float u = at[r] * 0.15915494f;
      u = u - rintf(u);
      cv[r] = __builtin_amdgcn_cosf(u) * 1.1f;
      sv[r] = __builtin_amdgcn_sinf(u) * 1.1f;
    }
    __builtin_amdgcn_sched_barrier(0);
    f4 c = z4, s = z4;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      c = MF(x, cv[r], c);
      s = MF(y, sv[r], s);
    }
    s1 += c[0] + s[2];
  }
  __builtin_amdgcn_sched_barrier(0);
  unsigned long long t5 = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
  {  // F: two independent 2-MFMA tiles, batched trans for both, then 8+8 MFMAs
    f4 at = MF(x, s1, z4), bt = MF(s1, y, z4);
    at = MF(y, s1, at);
    bt = MF(s1, x, bt);
    float cv[4], sv[4], cw[4], sw[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float u = at[r] * 0.15915494f, w = bt[r] * 0.15915494f;
      u = u - rintf(u);
      w = w - rintf(w);
      cv[r] = __builtin_amdgcn_cosf(u) * 1.1f;
      sv[r] = __builtin_amdgcn_sinf(u) * 1.1f;
      cw[r] = __builtin_amdgcn_cosf(w) * 1.1f;
      sw[r] = __builtin_amdgcn_sinf(w) * 1.1f;
    }
    __builtin_amdgcn_sched_barrier(0);
    f4 c = z4, s = z4, c2 = z4, s2 = z4;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      c = MF(x, cv[r], c);
      s = MF(y, sv[r], s);
      c2 = MF(cw[r], x, c2);
      s2 = MF(sw[r], y, s2);
    }
    s1 += c[0] + s[2] + c2[1] + s2[3];
  }
  __builtin_amdgcn_sched_barrier(0);
  unsigned long long t6 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x + blockIdx.x * 256] = s0 + s1;
  if (lane == 0 && threadIdx.x == 0) {
    t[blockIdx.x * 4 + 0] = t1 - t0;
    t[blockIdx.x * 4 + 1] = t2 - t1;
    t[blockIdx.x * 4 + 2] = t3 - t2;
    t[blockIdx.x * 4 + 3] = t4 - t3;
    t[G_ * 4 + blockIdx.x * 2 + 0] = t5 - t4;
    t[G_ * 4 + blockIdx.x * 2 + 1] = t6 - t5;
  }
}

int main() {
  const int G = 256;
  float *in, *out;
  unsigned long long* t;
  hipMalloc(&in, 512 * 4);
  hipMalloc(&out, G * 256 * 4);
  hipMalloc(&t, G * 6 * 8);
  std::vector<float> h(512);
  for (int i = 0; i < 512; ++i) h[i] = 0.001f * (i % 97);
  hipMemcpy(in, h.data(), 512 * 4, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(k, dim3(G), dim3(256), 0, 0, in, out, t);
  hipDeviceSynchronize();
  std::vector<unsigned long long> ht(G * 6);
  hipMemcpy(ht.data(), t, G * 6 * 8, hipMemcpyDeviceToHost);
  const char* names[4] = {"A 8 indep MFMA", "B 8 dependent MFMA", "C feature pattern (2+8 MFMA, 8 trans)",
                          "D feature pattern, VALU tail"};
  for (int j = 0; j < 4; ++j) {
    std::vector<unsigned long long> v(G);
    for (int i = 0; i < G; ++i) v[i] = ht[i * 4 + j];
    std::sort(v.begin(), v.end());
    printf("%-42s median %llu cycles (min %llu)\n", names[j], v[G / 2], v[0]);
  }
  const char* n2[2] = {"E C with trans batched before MFMAs", "F two tiles, batched, 16 MFMAs"};
  for (int j = 0; j < 2; ++j) {
    std::vector<unsigned long long> v(G);
    for (int i = 0; i < G; ++i) v[i] = ht[G * 4 + i * 2 + j];
    std::sort(v.begin(), v.end());
    printf("%-42s median %llu cycles (min %llu)\n", n2[j], v[G / 2], v[0]);
  }
  return 0;
}
