// misc_kernels.hip — parameter construction, initial draws and the RMSprop preconditioner.
#include "dgprf_internal.h"

namespace {

// N(0,1) fill from Philox (replaces tf.random.normal at layers/rf_layers.py:22,
// layers/GP_weight_layers.py:9, models/dgp.py:240).  One thread per counter quad.
__global__ void k_philox_normal(float* __restrict__ out, const int64_t n, const uint64_t seed,
                                const uint64_t sub, const uint32_t purpose) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t e0 = 4 * q;
  if (e0 >= n) return;
  const f4 z = philox_normal4(seed, sub, purpose, 0u, (uint32_t)q);
#pragma unroll
  for (int r = 0; r < 4; ++r)
    if (e0 + r < n) out[e0 + r] = z[r];
}

// Omega_l = exp(log_inv_ls_l)[:, None] * z_l + mean_l   (layers/rf_layers.py:34-38,
// kernels/RBF.py:51-53); c_l (rf_layers.py:44 / :90) and sigma^2 (likelihoods/gaussian.py:14-16).
__global__ void k_omega_build(const dgprf_plan_t pl, const float* __restrict__ z,
                              const float* __restrict__ hyp, float* __restrict__ omega,
                              float* __restrict__ der) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (pl.hyp_per_chain) {  // chain blockIdx.y: its own hyper-parameters (full_bayesian=True)
    hyp += (int64_t)blockIdx.y * pl.hyp_total;
    omega += (int64_t)blockIdx.y * pl.omega_total;
    der += (int64_t)blockIdx.y * pl.der_total;
  }
  if (i == 0) {
    for (int l = 0; l < pl.n_layers; ++l) {
      const float amp = expf(hyp[l]);
      const float sq = sqrtf((float)pl.n_rf[l]);
      der[l] = pl.kind[l] == DGPRF_RBF ? amp / sq : (sqrtf(2.f) * amp) / sq;
    }
    der[DGPRF_MAX_LAYERS] = expf(hyp[pl.n_layers]);
  }
  if (i >= pl.omega_total) return;
  int layer = 0;
  for (int l = 1; l < pl.n_layers; ++l)
    if (i >= pl.omega_off[l]) layer = l;
  const int64_t j = i - pl.omega_off[layer];
  const int k = (int)(j / pl.n_rf[layer]);
  const float ils = expf(hyp[pl.lis_off[layer] + k]);
  omega[i] = ils * z[i] + hyp[pl.mean_off[layer] + k];
}

// Stand-alone layer: Omega = exp(lis)[:,None] z + mean[:,None]; c.
__global__ void k_rf_omega(const int kind, const int d, const int R, const float* __restrict__ z,
                           const float* __restrict__ lis, const float* __restrict__ mean,
                           const float* __restrict__ log_amp, float* __restrict__ omega,
                           float* __restrict__ c) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) {
    const float amp = expf(*log_amp);
    const float sq = sqrtf((float)R);
    *c = kind == DGPRF_RBF ? amp / sq : (sqrtf(2.f) * amp) / sq;
  }
  if (i >= (int64_t)d * R) return;
  const int k = (int)(i / R);
  omega[i] = expf(lis[k]) * z[i] + mean[k];
}

// Welford step (models/dgp.py:268-271) on every W element of every chain.
__global__ void k_welford(const int64_t total, const float* __restrict__ grad,
                          float* __restrict__ mean, float* __restrict__ m2, const int k) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const float g = grad[i];
  const float mu = mean[i];
  const float delta = g - mu;
  const float mu1 = mu + delta / (float)k;
  const float delta2 = g - mu1;
  mean[i] = mu1;
  m2[i] = m2[i] + delta * delta2;
}

// sqrt(mean over [base, base + cnt) of E[g^2] (or Var[g]) + 1e-7)  (models/dgp.py:276-288)
__device__ float mass_of(const float* __restrict__ mean, const float* __restrict__ m2,
                         int64_t base, int64_t cnt, int K, int centered, float* red) {
  float a = 0.f;
  for (int64_t i = threadIdx.x; i < cnt; i += blockDim.x) {
    const float v = centered ? m2[base + i] / (float)(K - 1)
                             : mean[base + i] * mean[base + i] + m2[base + i] / (float)K;
    a += v;
  }
  red[threadIdx.x] = a;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  return sqrtf(red[0] / (float)cnt + 1.0e-7f);
}

// mass of W_l: block per (chain, layer); cs = chain stride of mean / m2
__global__ __launch_bounds__(256) void k_mass(const dgprf_plan_t pl, const float* __restrict__ mean,
                                              const float* __restrict__ m2, const int K,
                                              const int centered, const int64_t cs,
                                              float* __restrict__ mass) {
  __shared__ float red[256];
  const int layer = blockIdx.x, chain = blockIdx.y;
  const int64_t cnt = (int64_t)pl.P[layer] * pl.n_gp[layer];
  const float m = mass_of(mean, m2, (int64_t)chain * cs + pl.w_off[layer], cnt, K, centered, red);
  if (threadIdx.x == 0) mass[chain * pl.n_layers + layer] = m;
}

// masses of the trainable hyper-parameter variables (full_bayesian=True), block per
// (DGPRF_HMASS slot, chain); the hyper gradients follow W in the [w_total + hyp_total] layout.
__global__ __launch_bounds__(256) void k_hmass(const dgprf_plan_t pl, const float* __restrict__ mean,
                                               const float* __restrict__ m2, const int K,
                                               const int centered, float* __restrict__ hmass) {
  __shared__ float red[256];
  const int slot = blockIdx.x, chain = blockIdx.y, L = pl.n_layers;
  const int64_t base = (int64_t)chain * (pl.w_total + pl.hyp_total) + pl.w_total;
  const bool kern = (pl.hyp_flags & DGPRF_HYP_KERNEL) != 0, mn = (pl.hyp_flags & DGPRF_HYP_MEAN) != 0;
  const bool lik = (pl.hyp_flags & DGPRF_HYP_LIK) != 0 && pl.likelihood == DGPRF_LIK_GAUSSIAN;
  int64_t off = -1, cnt = 0;
  if (slot < 8 && slot < L && kern) {
    off = slot;  // log_amp
    cnt = 1;
  } else if (slot >= 8 && slot < 16 && slot - 8 < L && kern) {
    const int l = slot - 8;  // log_inv_ls: d_l slots, or one scalar
    off = pl.lis_off[l];
    cnt = pl.ard[l] ? pl.d[l] : 1;
  } else if (slot >= 16 && slot < 24 && slot - 16 < L && mn) {
    const int l = slot - 16;
    off = pl.mean_off[l];
    cnt = pl.d[l];
  } else if (slot == 24 && lik) {
    off = L;  // lik_log_var
    cnt = 1;
  }
  float m = 0.f;
  if (off >= 0) m = mass_of(mean, m2, base + off, cnt, K, centered, red);
  if (threadIdx.x == 0) hmass[chain * DGPRF_HMASS + slot] = m;
}

}  // namespace

namespace dgprf {

hipError_t launch_philox_normal(float* out, int64_t n, uint64_t seed, uint64_t sub,
                                uint32_t purpose, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int64_t quads = (n + 3) / 4;
  hipLaunchKernelGGL(k_philox_normal, dim3((unsigned)((quads + 255) / 256)), dim3(256), 0, s, out, n,
                     seed, sub, purpose);
  return hipGetLastError();
}

hipError_t launch_omega_build(const dgprf_plan_t& pl, const float* z, const float* hyp,
                              float* omega, float* der, hipStream_t s) {
  const int64_t n = pl.omega_total > 0 ? pl.omega_total : 1;
  hipLaunchKernelGGL(k_omega_build,
                     dim3((unsigned)((n + 255) / 256), pl.hyp_per_chain ? pl.n_chains : 1),
                     dim3(256), 0, s, pl, z, hyp, omega, der);
  return hipGetLastError();
}

hipError_t launch_rf_omega(int kind, int d, int R, const float* z, const float* lis,
                           const float* mean, const float* log_amp, float* omega, float* c,
                           hipStream_t s) {
  const int64_t n = (int64_t)d * R;
  hipLaunchKernelGGL(k_rf_omega, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, kind, d, R, z,
                     lis, mean, log_amp, omega, c);
  return hipGetLastError();
}

hipError_t launch_welford(const dgprf_plan_t& pl, const float* grad, float* mean, float* m2, int k,
                          bool full_bayes, hipStream_t s) {
  const int64_t total = (pl.w_total + (full_bayes ? pl.hyp_total : 0)) * pl.n_chains;
  hipLaunchKernelGGL(k_welford, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, total, grad,
                     mean, m2, k);
  return hipGetLastError();
}

hipError_t launch_mass_estimate(const dgprf_plan_t& pl, const float* mean, const float* m2, int K,
                                int centered, bool full_bayes, float* mass_est, float* hmass_est,
                                hipStream_t s) {
  const int64_t cs = pl.w_total + (full_bayes ? pl.hyp_total : 0);
  hipLaunchKernelGGL(k_mass, dim3(pl.n_layers, pl.n_chains), dim3(256), 0, s, pl, mean, m2, K,
                     centered, cs, mass_est);
  if (full_bayes)
    hipLaunchKernelGGL(k_hmass, dim3(DGPRF_HMASS, pl.n_chains), dim3(256), 0, s, pl, mean, m2, K,
                       centered, hmass_est);
  return hipGetLastError();
}

}  // namespace dgprf
