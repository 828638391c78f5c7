// launch_floor.hip — what does one dependent "phase" cost on MI355X?  Used to choose between
// kernel-per-phase (hipGraph) and a persistent kernel with in-launch barriers for the 7-phase
// SGHMC step.  Each phase: every thread loads 16 values written by the previous
// phase (a partial-sum consumer) and writes one value.
//   A: hipGraph of S steps x 7 kernels (grid 13x16 WGs of 256 threads, like the step kernels)
//   B: one persistent kernel, G resident WGs, 7 phases per step separated by a counter barrier
//      (agent release before arrive, relaxed polling with s_sleep, agent acquire after).
//   C: like B, but the cross-workgroup data itself moves with agent-scope relaxed atomic loads /
//      stores (coherent without L2 writeback / invalidate) and the barrier has no fences: stores
//      drained with s_waitcnt vmcnt(0) before the arrive.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CHECK(x)                                                               \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);         \
      return 1;                                                                \
    }                                                                          \
  } while (0)

constexpr int NPH = 7;
constexpr int SLOTS = 4096;

__global__ void k_phase(float* buf, int phase) {
  const float* src = buf + (size_t)(phase % 2) * SLOTS * 16;
  float* dst = buf + (size_t)((phase + 1) % 2) * SLOTS * 16;
  const int i = (blockIdx.y * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x;
  float v[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) v[s] = src[((i * 7 + s * 131) % SLOTS) * 16 + s];
  float a = 0.f;
#pragma unroll
  for (int s = 0; s < 16; ++s) a += v[s];
  if ((i & 15) == 0) dst[(i >> 4) % SLOTS * 16 + (i & 15)] = a * 0.5f + 1.f;
}

__device__ __forceinline__ void grid_sync(unsigned* ctr, unsigned target, unsigned* tmo) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 24)) {
        *tmo = 1;
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void k_persistent(float* buf, unsigned* ctr, unsigned* tmo,
                                                    int steps, int work_blocks) {
  const unsigned G = gridDim.x;
  unsigned phase_no = 0;
  for (int st = 0; st < steps; ++st) {
    for (int ph = 0; ph < NPH; ++ph) {
      const float* src = buf + (size_t)(ph % 2) * SLOTS * 16;
      float* dst = buf + (size_t)((ph + 1) % 2) * SLOTS * 16;
      for (int wb = blockIdx.x; wb < work_blocks; wb += G) {
        const int i = wb * blockDim.x + threadIdx.x;
        float v[16];
#pragma unroll
        for (int s = 0; s < 16; ++s) v[s] = src[((i * 7 + s * 131) % SLOTS) * 16 + s];
        float a = 0.f;
#pragma unroll
        for (int s = 0; s < 16; ++s) a += v[s];
        if ((i & 15) == 0) dst[(i >> 4) % SLOTS * 16 + (i & 15)] = a * 0.5f + 1.f;
      }
      ++phase_no;
      grid_sync(ctr, phase_no * G, tmo);
      if (*(volatile unsigned*)tmo) return;
    }
  }
}

__device__ __forceinline__ void grid_sync_light(unsigned* ctr, unsigned target, unsigned* tmo) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 24)) {
        *tmo = 1;
        break;
      }
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void k_persistent_light(float* buf, unsigned* ctr, unsigned* tmo,
                                                          int steps, int work_blocks) {
  const unsigned G = gridDim.x;
  unsigned phase_no = 0;
  for (int st = 0; st < steps; ++st) {
    for (int ph = 0; ph < NPH; ++ph) {
      float* src = buf + (size_t)(ph % 2) * SLOTS * 16;
      float* dst = buf + (size_t)((ph + 1) % 2) * SLOTS * 16;
      for (int wb = blockIdx.x; wb < work_blocks; wb += G) {
        const int i = wb * blockDim.x + threadIdx.x;
        float v[16];
#pragma unroll
        for (int s = 0; s < 16; ++s)
          v[s] = __hip_atomic_load(src + ((i * 7 + s * 131) % SLOTS) * 16 + s, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        float a = 0.f;
#pragma unroll
        for (int s = 0; s < 16; ++s) a += v[s];
        if ((i & 15) == 0)
          __hip_atomic_store(dst + (i >> 4) % SLOTS * 16 + (i & 15), a * 0.5f + 1.f,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      ++phase_no;
      grid_sync_light(ctr, phase_no * G, tmo);
      if (__hip_atomic_load(tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    }
  }
}

int main() {
  float* buf;
  unsigned *ctr, *tmo;
  CHECK(hipMalloc(&buf, 2 * SLOTS * 16 * sizeof(float)));
  CHECK(hipMalloc(&ctr, 256));
  CHECK(hipMalloc(&tmo, 256));
  CHECK(hipMemset(buf, 0, 2 * SLOTS * 16 * sizeof(float)));
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int S = 200;

  // ---- A: graph of S steps x 7 kernels
  for (int gx : {13, 1}) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int st = 0; st < S; ++st)
      for (int ph = 0; ph < NPH; ++ph)
        hipLaunchKernelGGL(k_phase, dim3(gx, gx == 13 ? 16 : 1), dim3(256), 0, s, buf, ph);
    CHECK(hipStreamEndCapture(s, &g));
    CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CHECK(hipGraphLaunch(ge, s));
    CHECK(hipStreamSynchronize(s));
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      CHECK(hipEventRecord(e0, s));
      CHECK(hipGraphLaunch(ge, s));
      CHECK(hipEventRecord(e1, s));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    printf("A graph  grid=%3d WGs : %.2f us/step  (%.2f us/phase)\n", gx == 13 ? 208 : 1,
           best * 1e3 / S, best * 1e3 / S / NPH);
    CHECK(hipGraphExecDestroy(ge));
    CHECK(hipGraphDestroy(g));
  }

  // ---- B: persistent kernel with in-launch barriers
  for (int G : {208, 128, 64, 32, 16}) {
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      CHECK(hipMemsetAsync(ctr, 0, 256, s));
      CHECK(hipMemsetAsync(tmo, 0, 256, s));
      CHECK(hipEventRecord(e0, s));
      hipLaunchKernelGGL(k_persistent, dim3(G), dim3(256), 0, s, buf, ctr, tmo, S, 208);
      CHECK(hipEventRecord(e1, s));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      unsigned h_tmo = 0;
      CHECK(hipMemcpy(&h_tmo, tmo, 4, hipMemcpyDeviceToHost));
      if (h_tmo) {
        printf("B persistent G=%d: barrier timeout\n", G);
        return 2;
      }
      best = ms < best ? ms : best;
    }
    printf("B persistent G=%3d WGs : %.2f us/step  (%.2f us/phase)\n", G, best * 1e3 / S,
           best * 1e3 / S / NPH);
  }
  // ---- C: persistent kernel, coherent data accesses, fence-free barrier
  for (int G : {208, 64, 16}) {
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      CHECK(hipMemsetAsync(ctr, 0, 256, s));
      CHECK(hipMemsetAsync(tmo, 0, 256, s));
      CHECK(hipEventRecord(e0, s));
      hipLaunchKernelGGL(k_persistent_light, dim3(G), dim3(256), 0, s, buf, ctr, tmo, S, 208);
      CHECK(hipEventRecord(e1, s));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      unsigned h_tmo = 0;
      CHECK(hipMemcpy(&h_tmo, tmo, 4, hipMemcpyDeviceToHost));
      if (h_tmo) {
        printf("C light G=%d: barrier timeout\n", G);
        return 2;
      }
      best = ms < best ? ms : best;
    }
    printf("C light  G=%3d WGs : %.2f us/step  (%.2f us/phase)\n", G, best * 1e3 / S,
           best * 1e3 / S / NPH);
  }
  return 0;
}
