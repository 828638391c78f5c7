// dgprf_internal.h — launcher declarations shared by the .hip translation units of libdgprf.so.
#pragma once
#include <hip/hip_runtime.h>

#include "dgprf_device.h"

// Everything a step kernel needs besides the plan (passed by value as a kernel argument).
struct StepDev {
  float* theta;
  float* mom;
  float* omega;
  float* der;
  const float* mass;
  float* ws;
  const int64_t* step;
  float* grad_out;  // grad_only mode: [C][w_total] (full_bayes: [C][w_total + hyp_total])
  uint64_t seed;
  BatchDev bd;
  int32_t step_offset;
  int32_t full_bayes;
  // chain strides of omega / der / hyp (0 = shared by the chains)
  int64_t om_cs, der_cs, hyp_cs;
  // full_bayesian=True state
  const float* z;
  float* hyp;
  float* hmom;
  const float* hmass;
};

struct UpdateDev {
  float lr, beta, temperature, data_size;
  int32_t resample, schedule, grad_only, resample_head;
  int64_t start_step, cycle_length;
  const float* xi;
  const float* xi_resample;
  const float* xi_hyp;
  const float* xi_hyp_resample;
};

// In-kernel timestamps for a separate diagnostic build (-DDGPRF_STAMPS); never in the product.
// The stamp array lives in the translation unit that defines DGPRF_STAMPS_TU (step_kernels.hip:
// the update kernel); the other units' stamps compile to nothing (no -fgpu-rdc across units).
#if defined(DGPRF_STAMPS) && defined(DGPRF_STAMPS_TU)
extern __device__ unsigned long long g_dgprf_stamps[];
#define DGPRF_STAMP_SLOTS 16
#define DGPRF_STAMP_BASES (17 * 4096)
#define DGPRF_STAMP(base, i)                                                      \
  do {                                                                           \
    if (threadIdx.x == 0 && (size_t)(base) < DGPRF_STAMP_BASES) {                \
      __builtin_amdgcn_sched_barrier(0);                                         \
      g_dgprf_stamps[(size_t)(base) * DGPRF_STAMP_SLOTS + (i)] =                 \
          __builtin_amdgcn_s_memtime();                                          \
      if ((i) == 0)                                                              \
        g_dgprf_stamps[(size_t)(base) * DGPRF_STAMP_SLOTS + 15] =                \
            __builtin_amdgcn_s_memrealtime();                                    \
      if ((i) == 14)                                                             \
        g_dgprf_stamps[(size_t)(base) * DGPRF_STAMP_SLOTS + 13] =                \
            __builtin_amdgcn_s_memrealtime();                                    \
      __builtin_amdgcn_sched_barrier(0);                                         \
    }                                                                            \
  } while (0)
// per-wave placement: slots 8..11 = HW_ID | XCC_ID << 32 of waves 0..3
#define DGPRF_STAMP_HWID(base)                                                   \
  do {                                                                           \
    if ((threadIdx.x & 63) == 0 && threadIdx.x < 256 &&                          \
        (size_t)(base) < DGPRF_STAMP_BASES) {                                    \
      const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);  \
      const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20);\
      g_dgprf_stamps[(size_t)(base) * DGPRF_STAMP_SLOTS + 8 + (threadIdx.x >> 6)] = \
          (unsigned long long)hw | ((unsigned long long)xcc << 32);              \
    }                                                                            \
  } while (0)
#else
#define DGPRF_STAMP_HWID(base) \
  do {                         \
  } while (0)
#define DGPRF_STAMP(base, i) \
  do {                       \
    (void)(base);            \
  } while (0)
#endif

namespace dgprf {
// Dynamic LDS above 64 KiB must be opted into per kernel.
inline void set_lds_limit(const void* fn, size_t bytes) {
  if (bytes > 65536) (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

// Forward / backward of one layer of the step (k_step_fwd / k_step_bwd).
// with_agemm = false: layer 0 without its A_1 = X Omega_1 GEMM (timed apart by dgprf_profile_step)
hipError_t launch_step_fwd(const dgprf_plan_t& pl, const StepDev& sd, int layer, hipStream_t s,
                           bool with_agemm = true);
hipError_t launch_step_bwd(const dgprf_plan_t& pl, const StepDev& sd, int layer, hipStream_t s);
// Large minibatches, one chain (dgprf_sk::step_fused_fwd): the forward of every layer as one
// launch of the predictive kernel, complete F_l into slice 0 of the F partial buffers.
hipError_t launch_step_fwd_fused(const dgprf_plan_t& pl, const StepDev& sd, hipStream_t s);
// Sums the gW partials, adds the prior term and applies the SGHMC update (or writes the gradient);
// gather_next: extra workgroups gather step t+1's minibatch rows.
hipError_t launch_step_update(const dgprf_plan_t& pl, const StepDev& sd, const UpdateDev& ud,
                              const float* grad_in, hipStream_t s, bool gather_next = false,
                              bool advance = false);
// (sd.full_bayes: the same launch also runs the hyper-parameter workgroups — their gradients or
// update and the Omega, c, sigma^2 rebuild)

// minibatch rows of step *step + step_offset into the workspace (no-op for DGPRF_BATCH_DIRECT)
hipError_t launch_gather(const dgprf_plan_t& pl, const StepDev& sd, hipStream_t s);
// A = X Omega for n rows (X row stride ld, K = d), written [align32(n)][R]: the wide-first-layer GEMM
hipError_t launch_agemm(const float* X, int64_t n, int ld, int d, const float* om, int R,
                        float* aout, hipStream_t s);
hipError_t launch_advance(int64_t* step, int64_t by, hipStream_t s);
// The step's A_1 GEMM alone (plan.a0_off >= 0): the hand-written MFMA kernel of agemm.hip.
hipError_t launch_step_agemm(const dgprf_plan_t& pl, const StepDev& sd, hipStream_t s);
// The hand-written MFMA A_1 GEMM (agemm.hip): A[n_out][R] = X[n][d] Omega[d][R] (rows >= n
// zero) for `batch` chains (element strides sx, so, sa; so = 0: shared Omega).  parts = 2: two
// K-part slabs sp floats apart whose sum is A (the step's layer-0 consumers add them); parts = 1:
// A whole.  false: shape outside the kernel (d, ldx, R not multiples of 4, or too large for
// 32-bit offsets).
bool own_agemm(const float* X, int64_t n, int64_t n_out, int ldx, int d, const float* om, int R,
               float* aout, int batch, int64_t sx, int64_t so, int64_t sa, int parts, int64_t sp,
               hipStream_t s, hipError_t* err);
bool agemm_shape_ok(int64_t n, int64_t n_out, int ldx, int d, int R);
// K parts the step's A_1 GEMM writes (2 for step-sized row counts the kernel takes, else 1)
int agemm_parts(int64_t n, int64_t n_out, int ldx, int d, int R);
// plan.fresh_z: Omega of every layer into the workspace (omf_off), fresh layers from Philox z of
// step *step + step_offset, the others copied from the chain's Omega when the all-layer fused
// forward reads this copy (per-layer kernels read a fixed layer's Omega in place)
hipError_t launch_fresh_omega(const dgprf_plan_t& pl, const StepDev& sd, hipStream_t s);

// How dgprf_forward covers n rows: tile or row kernel, the A_1 GEMM for a wide first layer (in
// row chunks of `chunk` rows of caller scratch).  Host-only, shared by the launcher and the
// scratch query so both size the chunks identically.
struct ForwardCfg {
  bool wide0, tiles;
  int rows_waves;  // waves per workgroup of the row kernel (4, 8 or 16)
  int rows_tt;     // 16-row tiles per row-kernel workgroup (2: one sample, tiles outnumber the CUs)
  int64_t chunk, scratch_floats;
};
// n_samples: posterior samples scored by one launch (grid.z); the path choice counts all its rows
ForwardCfg forward_cfg(const dgprf_plan_t& pl, int64_t n, int n_samples = 1);
hipError_t launch_forward_rows(const dgprf_plan_t& pl, const float* theta, const float* omega,
                               const float* der, const float* X, const float* Y, int y_cols,
                               int64_t n, float* const* f_out, float* logp, float* se,
                               float* lse_m, float* lse_s, float* se_sum, float* scratch,
                               hipStream_t s, const float* a1_full = nullptr, int n_samples = 1,
                               int path_samples = 0);
// (a1_full: X Omega_1 of all n rows, precomputed by the caller for a wide first layer: no A_1 GEMM;
// path_samples > 0: choose the kernel as for a launch of that many samples — the per-sample
// launches of a multi-sample call take the kernel its one-launch form takes, so both agree bitwise)
// Posterior-predictive LSE fold of n_samples samples of every chain (thetas [n_samples][C][w_total]),
// sample order: two samples per pass of the pair kernel for lean models (layer 0 shared) — every
// pair in one launch when scratch holds forward_samples_scratch floats — else one
// launch_forward_rows per sample.
hipError_t launch_forward_samples(const dgprf_plan_t& pl, const float* thetas, int n_samples,
                                  const float* omega, const float* der, const float* X,
                                  const float* A1, const float* Y, int y_cols, int64_t n, float* lse_m,
                                  float* lse_s, float* se_sum, float* scratch,
                                  int64_t scratch_floats, hipStream_t s);
bool forward_pairs_ok(const dgprf_plan_t& pl, int64_t n, int n_samples = 1);
// scratch floats that let launch_forward_samples run every pair in one launch (0: not applicable)
int64_t forward_samples_scratch(const dgprf_plan_t& pl, int64_t n, int n_samples);
hipError_t launch_lse_finalize(const float* lse_m, const float* lse_s, const float* se_sum,
                               int parts, int64_t n, double s_total, float log_y_std, float y_std,
                               float* lse_out, double* out, hipStream_t s);
hipError_t launch_rf_features(int kind, const float* X, int64_t n, int d, const float* omega,
                              int R, const float* c, float* phi, hipStream_t s);
hipError_t launch_gp_matmul(const float* phi, int64_t n, int P, const float* W, int g, float* F,
                            hipStream_t s);
hipError_t launch_prior_w(const dgprf_plan_t& pl, const float* theta, float* out, hipStream_t s);

hipError_t launch_philox_normal(float* out, int64_t n, uint64_t seed, uint64_t sub,
                                uint32_t purpose, hipStream_t s);
// Omega / c / sigma^2 of every chain when pl.hyp_per_chain (chain strides omega_total, der_total,
// hyp_total), else the shared copy.
hipError_t launch_omega_build(const dgprf_plan_t& pl, const float* z, const float* hyp,
                              float* omega, float* der, hipStream_t s);
hipError_t launch_rf_omega(int kind, int d, int R, const float* z, const float* lis,
                           const float* mean, const float* log_amp, float* omega, float* c,
                           hipStream_t s);
hipError_t launch_welford(const dgprf_plan_t& pl, const float* grad, float* mean, float* m2, int k,
                          bool full_bayes, hipStream_t s);
hipError_t launch_mass_estimate(const dgprf_plan_t& pl, const float* mean, const float* m2, int K,
                                int centered, bool full_bayes, float* mass_est, float* hmass_est,
                                hipStream_t s);
}  // namespace dgprf
