// mfma_rates.hip — diagnostic: cycles per f32 MFMA on one wave (s_memtime around an unrolled loop)
// for the forms the kernels use: 4x4x1_16b (predictive F contraction, g <= 8), 16x16x4 and
// 32x32x2, each with 1 (dependent chain) and 4 / 8 independent accumulators, and the 4x4x1 form
// interleaved with v_sin/v_cos as in the predictive chunk body.  Not product code.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o mfma_rates mfma_rates.hip && ./mfma_rates
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

#define CK(x)                                                        \
  do {                                                               \
    if ((x) != hipSuccess) {                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, #x);         \
      return 1;                                                      \
    }                                                                \
  } while (0)

constexpr int ITERS = 256;

template <int FORM, int NACC, int TRIG>
__global__ __launch_bounds__(64) void k_rate(const float* in, float* out, unsigned long long* cyc) {
  float a = in[threadIdx.x], b = in[64 + threadIdx.x];
  f4 c4[NACC];
  f16v c16[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) {
    c4[i] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 16; ++r) c16[i][r] = 0.f;
  }
  float t0 = a, t1 = b;
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long s0 = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) {
      if (FORM == 0) c4[i] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c4[i], 0, 0, 0);
      if (FORM == 1) c4[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c4[i], 0, 0, 0);
      if (FORM == 2) c16[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c16[i], 0, 0, 0);
      if (TRIG && (i % TRIG) == 0) {  // one sin + one cos (+ fract) per TRIG MFMAs
        const float u = __builtin_amdgcn_fractf(t0);
        t0 = __builtin_amdgcn_sinf(u) + t1;
        t1 = __builtin_amdgcn_cosf(u);
      }
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long s1 = __builtin_amdgcn_s_memtime();
  float acc = t0 + t1;
#pragma unroll
  for (int i = 0; i < NACC; ++i) {
    acc += c4[i][0] + c4[i][3];
    acc += c16[i][0] + c16[i][15];
  }
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[0] = s1 - s0;
}

template <int FORM, int NACC, int TRIG>
int run(const char* name, const float* in, float* out, unsigned long long* cyc) {
  hipLaunchKernelGGL((k_rate<FORM, NACC, TRIG>), dim3(1), dim3(64), 0, 0, in, out, cyc);
  hipLaunchKernelGGL((k_rate<FORM, NACC, TRIG>), dim3(1), dim3(64), 0, 0, in, out, cyc);
  CK(hipDeviceSynchronize());
  unsigned long long h = 0;
  CK(hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost));
  printf("%-44s %7.2f cycles per MFMA\n", name, (double)h / (ITERS * NACC));
  return 0;
}

// Two roles on each SIMD (waves w and w + 4 of a 512-thread workgroup share a SIMD): role 0 runs
// ITERS x 16 4x4x1_16b MFMAs (4 accumulators), role 1 runs ITERS x 16 independent fract + sin + cos
// (16 streams).  MODE 0: both roles MFMA; 1: MFMA | trig; 2: both trig; 3: MFMA | idle; 4: trig | idle.
template <int MODE>
__global__ __launch_bounds__(512) void k_mix(const float* in, float* out, unsigned long long* cyc) {
  const int wave = threadIdx.x >> 6, role = wave >= 4;
  const bool mfma = role == 0 ? (MODE != 2 && MODE != 4) : (MODE == 0);
  const bool trig = role == 0 ? (MODE == 2 || MODE == 4) : (MODE == 1 || MODE == 2);
  float a = in[threadIdx.x & 63], b = in[64 + (threadIdx.x & 63)];
  f4 c[4] = {};
  float t[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) t[i] = a + i;
  __syncthreads();
  const unsigned long long s0 = __builtin_amdgcn_s_memtime();
  if (mfma) {
    for (int it = 0; it < ITERS; ++it)
#pragma unroll
      for (int i = 0; i < 16; ++i) c[i & 3] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c[i & 3], 0, 0, 0);
  } else if (trig) {
    for (int it = 0; it < ITERS; ++it)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float u = __builtin_amdgcn_fractf(t[i]);
        t[i] = __builtin_amdgcn_sinf(u) + __builtin_amdgcn_cosf(u);
      }
  }
  const unsigned long long s1 = __builtin_amdgcn_s_memtime();
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc += t[i];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc += c[i][0];
  out[threadIdx.x] = acc;
  if ((threadIdx.x & 63) == 0) cyc[wave] = s1 - s0;
}

template <int MODE>
int run_mix(const char* name, const float* in, float* out, unsigned long long* cyc) {
  hipLaunchKernelGGL((k_mix<MODE>), dim3(1), dim3(512), 0, 0, in, out, cyc);
  hipLaunchKernelGGL((k_mix<MODE>), dim3(1), dim3(512), 0, 0, in, out, cyc);
  CK(hipDeviceSynchronize());
  unsigned long long h[8];
  CK(hipMemcpy(h, cyc, 64, hipMemcpyDeviceToHost));
  unsigned long long m0 = 0, m1 = 0;
  for (int w = 0; w < 4; ++w) m0 = h[w] > m0 ? h[w] : m0;
  for (int w = 4; w < 8; ++w) m1 = h[w] > m1 ? h[w] : m1;
  printf("%-44s role0 %7.2f  role1 %7.2f cycles per item (16 per iteration)\n", name,
         (double)m0 / (ITERS * 16), (double)m1 / (ITERS * 16));
  return 0;
}

int main() {
  float *in, *out;
  unsigned long long* cyc;
  CK(hipMalloc(&in, 128 * 4));
  CK(hipMalloc(&out, 512 * 4));
  CK(hipMalloc(&cyc, 64));
  CK(hipMemset(in, 0, 128 * 4));
  run<0, 1, 0>("4x4x1_16b  1 acc (dependent)", in, out, cyc);
  run<0, 2, 0>("4x4x1_16b  2 acc", in, out, cyc);
  run<0, 4, 0>("4x4x1_16b  4 acc", in, out, cyc);
  run<0, 8, 0>("4x4x1_16b  8 acc", in, out, cyc);
  run<0, 4, 1>("4x4x1_16b  4 acc + sin/cos per MFMA", in, out, cyc);
  run<0, 4, 2>("4x4x1_16b  4 acc + sin/cos per 2 MFMA", in, out, cyc);
  run<0, 4, 4>("4x4x1_16b  4 acc + sin/cos per 4 MFMA", in, out, cyc);
  run<1, 1, 0>("16x16x4    1 acc (dependent)", in, out, cyc);
  run<1, 2, 0>("16x16x4    2 acc", in, out, cyc);
  run<1, 4, 0>("16x16x4    4 acc", in, out, cyc);
  run<1, 4, 1>("16x16x4    4 acc + sin/cos per MFMA", in, out, cyc);
  run<2, 1, 0>("32x32x2    1 acc (dependent)", in, out, cyc);
  run<2, 4, 0>("32x32x2    4 acc", in, out, cyc);
  run_mix<3>("mix: 4x4x1 | idle", in, out, cyc);
  run_mix<4>("mix: trig | idle", in, out, cyc);
  run_mix<0>("mix: 4x4x1 | 4x4x1", in, out, cyc);
  run_mix<2>("mix: trig | trig", in, out, cyc);
  run_mix<1>("mix: 4x4x1 | trig", in, out, cyc);
  return 0;
}
