// mfma4x4.hip — operand/result layout and cycle costs of v_mfma_f32_4x4x1_16b_f32 on gfx950
// (no vendor documentation in this image; measured).
//   layout: A = lane code, B = 1  ->  D reveals which A lane feeds D[lane][reg];
//           A = 1, B = lane code  ->  which B lane feeds D[lane][reg]
//   cycles (one wave per SIMD, s_memtime, median over 256 workgroups):
//     T0: 32 independent 4x4x1_16b (4 accumulators)      T1: 32 dependent (one accumulator)
//     T2: 32 independent 16x16x4                         T3: 4x4 chain + 1 v_sin per MFMA
//     T4: per-chunk pattern of the predictive kernel with 4x4 blocks for g = 8
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
#define M4(a, b, c) __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0)
#define M16(a, b, c) __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0)

__global__ void k_layout(float* out) {
  const int lane = threadIdx.x;
  const f4 z = {0, 0, 0, 0};
  f4 da = M4((float)lane, 1.0f, z);
  f4 db = M4(1.0f, (float)lane, z);
  for (int r = 0; r < 4; ++r) {
    out[lane * 4 + r] = da[r];
    out[256 + lane * 4 + r] = db[r];
  }
}

#define STAMP(t)                             \
  __builtin_amdgcn_sched_barrier(0);         \
  t = __builtin_amdgcn_s_memtime();          \
  __builtin_amdgcn_sched_barrier(0);

__global__ __launch_bounds__(256) void k_cyc(const float* in, float* out, unsigned long long* t) {
  float x = in[threadIdx.x], y = in[threadIdx.x + 256];
  const f4 z4 = {0, 0, 0, 0};
  f4 a = z4, b = z4, c = z4, d = z4;
  unsigned long long t0, t1, t2, t3, t4, t5;
  __builtin_amdgcn_s_waitcnt(0);
  STAMP(t0);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a = M4(x, y, a);
    b = M4(y, x, b);
    c = M4(x, x, c);
    d = M4(y, y, d);
  }
  float s0 = a[0] + b[1] + c[2] + d[3];
  STAMP(t1);
#pragma unroll
  for (int i = 0; i < 32; ++i) a = M4(x + s0, y, a);
  float s1 = a[1];
  STAMP(t2);
  f4 e = z4, f = z4;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    e = M16(x, y + s1, e);
    f = M16(y, x, f);
  }
  float s2 = e[0] + f[1];
  STAMP(t3);
  f4 g = z4, h = z4;
  float u = s2;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    float sv = __builtin_amdgcn_sinf(u + (float)i);
    g = M4(x, sv, g);
    h = M4(sv, y, h);
  }
  float s3 = g[0] + h[1];
  STAMP(t4);
  {
    // one 16-feature chunk with g = 8: 2 A-tile MFMAs, 4 (fract, sin, cos), 16 4x4 MFMAs in 4 chains
    f4 at = M16(x, s3, z4);
    at = M16(y, s3, at);
    f4 c0 = z4, c1 = z4, s0_ = z4, s1_ = z4;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float v = __builtin_amdgcn_fractf(at[r]);
      const float cv = __builtin_amdgcn_cosf(v), sv = __builtin_amdgcn_sinf(v);
      c0 = M4(x, cv, c0);
      c1 = M4(y, cv, c1);
      s0_ = M4(x, sv, s0_);
      s1_ = M4(y, sv, s1_);
    }
    s3 += c0[0] + c1[1] + s0_[2] + s1_[3];
  }
  STAMP(t5);
  out[blockIdx.x * 256 + threadIdx.x] = s3;
  if (threadIdx.x == 0) {
    unsigned long long* o = t + blockIdx.x * 5;
    o[0] = t1 - t0;
    o[1] = t2 - t1;
    o[2] = t3 - t2;
    o[3] = t4 - t3;
    o[4] = t5 - t4;
  }
}

int main() {
  float* dout;
  hipMalloc(&dout, 512 * sizeof(float));
  hipLaunchKernelGGL(k_layout, dim3(1), dim3(64), 0, 0, dout);
  std::vector<float> h(512);
  hipMemcpy(h.data(), dout, 512 * sizeof(float), hipMemcpyDeviceToHost);
  printf("layout: lane: reg0..3 of D with A=lane,B=1 | with A=1,B=lane\n");
  for (int l = 0; l < 64; ++l)
    printf("%2d: %4.0f %4.0f %4.0f %4.0f | %4.0f %4.0f %4.0f %4.0f\n", l, h[4 * l], h[4 * l + 1],
           h[4 * l + 2], h[4 * l + 3], h[256 + 4 * l], h[256 + 4 * l + 1], h[256 + 4 * l + 2],
           h[256 + 4 * l + 3]);
  const int NB = 256;
  float *din, *dout2;
  unsigned long long* dt;
  hipMalloc(&din, 512 * sizeof(float));
  hipMalloc(&dout2, NB * 256 * sizeof(float));
  hipMalloc(&dt, NB * 5 * sizeof(unsigned long long));
  std::vector<float> hin(512);
  for (int i = 0; i < 512; ++i) hin[i] = 0.001f * (i % 97);
  hipMemcpy(din, hin.data(), 512 * sizeof(float), hipMemcpyHostToDevice);
  for (int it = 0; it < 3; ++it)
    hipLaunchKernelGGL(k_cyc, dim3(NB), dim3(256), 0, 0, din, dout2, dt);
  hipDeviceSynchronize();
  std::vector<unsigned long long> ht(NB * 5);
  hipMemcpy(ht.data(), dt, ht.size() * 8, hipMemcpyDeviceToHost);
  const char* names[5] = {"T0 32 indep 4x4x1_16b", "T1 32 dep 4x4x1_16b", "T2 32 indep 16x16x4",
                          "T3 16x(sin + 2 4x4)", "T4 chunk g=8 via 4x4"};
  for (int k = 0; k < 5; ++k) {
    std::vector<unsigned long long> v;
    for (int b = 0; b < NB; ++b) v.push_back(ht[b * 5 + k]);
    std::sort(v.begin(), v.end());
    printf("%-26s median %llu cycles (min %llu)\n", names[k], v[NB / 2], v[0]);
  }
  return 0;
}
