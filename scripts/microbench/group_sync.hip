// group_sync.hip — what does a dependent phase cost when the exchange is a ROW-TILE GROUP
// hand-off (16 workgroups) inside one persistent kernel, instead of a kernel boundary?
// The step's cross-workgroup sums are per row tile: F_l / dX_l slice partials of row tile rt are
// produced and consumed by the 16 feature-slice workgroups of rt only.
//   A: hipGraph of S steps x 7 kernels, 13 x 16 workgroups of 256 threads; each phase every
//      workgroup reads its row tile's 16 slice partials of the previous phase (16 rows x 8 floats
//      each) and writes its own.
//   D: one persistent kernel, same 208 workgroups and data flow; after each phase a workgroup
//      arrives on its row tile's counter (16 arrivals) and waits for it; the partials move with
//      agent-scope relaxed atomic stores / loads (coherent across XCDs without L2 maintenance).
//   E: D plus one grid-wide (two-level) barrier per step (the update needs every row tile).
// Every spin is bounded (timeout flag, the kernel then returns), and 208 workgroups of 256
// threads are co-resident on 256 CUs.
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHECK(x)                                                               \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);         \
      return 1;                                                                \
    }                                                                          \
  } while (0)

constexpr int NPH = 7, NRT = 13, NS = 16, ELEM = 16 * 8;  // floats per partial
constexpr unsigned SPIN_MAX = 1u << 22;

// partial buffer [2][NRT][NS][ELEM]
__device__ __forceinline__ float* part(float* buf, int ph, int rt, int s) {
  return buf + (((size_t)(ph & 1) * NRT + rt) * NS + s) * ELEM;
}

__global__ __launch_bounds__(256) void k_phase(float* buf, int ph) {
  const int rt = blockIdx.x / NS, s = blockIdx.x % NS, t = threadIdx.x;
  float acc = 0.f;
  if (t < ELEM) {
#pragma unroll
    for (int q = 0; q < NS; ++q) acc += part(buf, ph, rt, q)[t];
    part(buf, ph + 1, rt, s)[t] = acc * 0.0625f + 1.f;
  }
}

__device__ __forceinline__ bool wait_count(unsigned* ctr, unsigned target, unsigned* tmo) {
  unsigned spins = 0;
  while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
    __builtin_amdgcn_s_sleep(1);
    if (++spins > SPIN_MAX) {
      __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
  }
  return true;
}

template <bool GLOBAL>
__global__ __launch_bounds__(256) void k_persist(float* buf, unsigned* ctr, unsigned* tmo, int steps) {
  const int rt = blockIdx.x / NS, s = blockIdx.x % NS, t = threadIdx.x;
  unsigned* gctr = ctr + NRT * 32;  // grid counter (its own cache lines)
  unsigned n = 0, gn = 0;
  __shared__ int bad;
  for (int st = 0; st < steps; ++st) {
    for (int ph = 0; ph < NPH; ++ph) {
      float acc = 0.f;
      if (t < ELEM) {
#pragma unroll
        for (int q = 0; q < NS; ++q)
          acc += __hip_atomic_load(part(buf, ph, rt, q) + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(part(buf, ph + 1, rt, s) + t, acc * 0.0625f + 1.f, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      ++n;
      if (t == 0) {
        __hip_atomic_fetch_add(ctr + rt * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bad = !wait_count(ctr + rt * 32, n * NS, tmo);
      }
      __syncthreads();
      if (bad) return;
    }
    if (GLOBAL) {  // two-level: row-tile leaders arrive on the grid counter
      ++gn;
      if (t == 0) {
        bool ok = true;
        if (s == 0) __hip_atomic_fetch_add(gctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = wait_count(gctr, gn * NRT, tmo);
        bad = !ok;
      }
      __syncthreads();
      if (bad) return;
    }
  }
}

int main() {
  float* buf;
  unsigned *ctr, *tmo;
  const size_t nf = (size_t)2 * NRT * NS * ELEM;
  CHECK(hipMalloc(&buf, nf * sizeof(float)));
  CHECK(hipMalloc(&ctr, 4096));
  CHECK(hipMalloc(&tmo, 256));
  CHECK(hipMemset(buf, 0, nf * sizeof(float)));
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int S = 200, G = NRT * NS;

  {  // A: graph of kernels
    hipGraph_t g;
    hipGraphExec_t ge;
    CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int st = 0; st < S; ++st)
      for (int ph = 0; ph < NPH; ++ph) hipLaunchKernelGGL(k_phase, dim3(G), dim3(256), 0, s, buf, ph);
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
    printf("A graph of kernels      : %.2f us/step (%.2f us/phase)\n", best * 1e3 / S, best * 1e3 / S / NPH);
    CHECK(hipGraphExecDestroy(ge));
    CHECK(hipGraphDestroy(g));
  }
  for (int glob = 0; glob < 2; ++glob) {
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      CHECK(hipMemsetAsync(ctr, 0, 4096, s));
      CHECK(hipMemsetAsync(tmo, 0, 256, s));
      CHECK(hipEventRecord(e0, s));
      if (glob) hipLaunchKernelGGL(k_persist<true>, dim3(G), dim3(256), 0, s, buf, ctr, tmo, S);
      else hipLaunchKernelGGL(k_persist<false>, dim3(G), dim3(256), 0, s, buf, ctr, tmo, S);
      CHECK(hipEventRecord(e1, s));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      unsigned h = 0;
      CHECK(hipMemcpy(&h, tmo, 4, hipMemcpyDeviceToHost));
      if (h) {
        printf("%s: spin timeout\n", glob ? "E" : "D");
        return 2;
      }
      best = ms < best ? ms : best;
    }
    printf("%s persistent, row-tile groups%s: %.2f us/step (%.2f us/phase)\n", glob ? "E" : "D",
           glob ? " + grid barrier/step" : "", best * 1e3 / S, best * 1e3 / S / NPH);
  }
  return 0;
}
