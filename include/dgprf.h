/*
 * dgprf.h — C-ABI of the MI355X-native DGP-RF SGHMC/SGLD engine (libdgprf.so).
 *
 * The reference (shixinxing/DGP-RF-MCMC) has no FFI: its hot path is TensorFlow-eager Python
 * (models/dgp.py, layers/rf_layers.py, layers/GP_weight_layers.py, kernels/RBF.py,
 * kernels/arc_cosine.py, likelihoods/{gaussian,softmax}.py, utils.py).  The Python mirror of that API
 * (dgp-rf-mcmc_amd/{models,layers,kernels,likelihoods}, utils.py) binds these entry points with
 * ctypes.  Every entry point below names the reference code it replaces.
 *
 * Conventions
 *  - All tensors are device pointers (HBM), fp32, row-major, exactly the TF layout of the
 *    reference (models/dgp.py:118-127; layers/rf_layers.py:42-44; layers/GP_weight_layers.py:13).
 *  - `stream` is a hipStream_t passed as void* (NULL = legacy default stream).  Every call is
 *    asynchronous w.r.t. the host and enqueues on that stream only.
 *  - Return value: 0 on success, a negative DGPRF_E* code otherwise (dgprf_error_string()).
 *    Shape/config errors are detected on the host before anything is enqueued.
 *  - No torch types cross this boundary.
 */
#ifndef DGPRF_H
#define DGPRF_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DGPRF_ABI_VERSION 10

#define DGPRF_MAX_LAYERS 8
#define DGPRF_MAX_G 64        /* max latent GPs per layer (n_gp[l]) */
#define DGPRF_MAX_D 2048      /* max layer input width d_l */

/* kernel types: models/dgp.py:80-90 (kernel_type_list entries 'RBF' / 'ARC') */
#define DGPRF_RBF 0
#define DGPRF_ARC 1

/* likelihoods: likelihoods/gaussian.py:6-25, likelihoods/softmax.py:4-22 */
#define DGPRF_LIK_GAUSSIAN 0
#define DGPRF_LIK_SOFTMAX 1

/* minibatch source modes (dgprf_batch_t.mode) */
#define DGPRF_BATCH_DIRECT 0   /* rows 0..B-1 of X/Y are the batch (sgmcmc_update(X_batch, ...)) */
#define DGPRF_BATCH_INDEXED 1  /* batch row b of chain c is X[idx[c*B + b]] */
#define DGPRF_BATCH_EPOCH 2    /* per-epoch keyed Feistel permutation of [0,N), drop-remainder */

/* step-size schedules (dgprf_step_t.schedule) */
#define DGPRF_SCHED_CONST 0    /* lr, temperature, resample as given */
#define DGPRF_SCHED_CYCLICAL 1 /* experiments/utils_training.py:41-61 + utils.py:49-73 on device */

/* Philox stream purposes (counter word 3, bits 24..31) */
#define DGPRF_RNG_NOISE 1      /* xi in m += sqrt(2(1-b)TM) xi   (models/dgp.py:212) */
#define DGPRF_RNG_RESAMPLE 2   /* m ~ N(0,1) on resample          (models/dgp.py:210) */
#define DGPRF_RNG_Z 3          /* z ~ N(0,1) RF frequencies       (layers/rf_layers.py:22) */
#define DGPRF_RNG_W 4          /* W ~ N(0,1) GP weights           (layers/GP_weight_layers.py:9) */
#define DGPRF_RNG_MOMENTS 5    /* initial momenta                 (models/dgp.py:240) */
#define DGPRF_RNG_HYPER 6      /* xi of the hyper-parameter updates (full_bayesian=True) */
#define DGPRF_RNG_HYPER_RESAMPLE 7 /* resampled hyper-parameter momenta          */

/* Trainable hyper-parameter groups of full_bayesian=True (plan.hyp_flags; models/dgp.py:175-181,
 * 199-204): the kernels' log_amplitude and log_inv_length_scale (kernel_trainable,
 * kernels/RBF.py:39-41), the layer means (set_nonzero_mean, layers/rf_layers.py:23-26) and the
 * Gaussian lik_log_var (likelihoods/gaussian.py:12). */
#define DGPRF_HYP_KERNEL 1
#define DGPRF_HYP_LIK 2
#define DGPRF_HYP_MEAN 4
/* Hyper-parameter masses per chain (dgprf_chain_t.hmass [C][DGPRF_HMASS]): log_amp of layer l at
 * l, log_inv_ls at 8 + l, mean at 16 + l, lik_log_var at 24 (one mass per tf.Variable, like the
 * reference's param.M). */
#define DGPRF_HMASS 32

/* predictive forward path (dgprf_plan_t.fwd_path).  AUTO is the product choice; the other two pin a
 * path for parity tests: the general row kernel, or a wide first layer contracted inside the forward
 * kernel instead of by the separate A_1 = X Omega_1 GEMM. */
#define DGPRF_FWD_AUTO 0
#define DGPRF_FWD_ROWS 1        /* row kernel, 4 waves per 16-row tile */
#define DGPRF_FWD_NO_AGEMM 2
#define DGPRF_FWD_TILE 3        /* tile kernel (one wave per 16-row tile) whatever the row count */
#define DGPRF_FWD_ROWS16 4      /* row kernel, 16 waves per 16-row tile (small test sets) */
#define DGPRF_FWD_ROWS8 5       /* row kernel, 8 waves per 16-row tile (two workgroups per CU) */

/* error codes */
#define DGPRF_OK 0
#define DGPRF_E_ARG -1         /* null pointer / bad scalar argument */
#define DGPRF_E_SHAPE -2       /* unsupported shape (layers, widths, batch) */
#define DGPRF_E_HIP -3         /* a HIP runtime call failed */
#define DGPRF_E_PLAN -4        /* plan not initialised by dgprf_plan_init */

/*
 * Model plan.  Caller fills the first block (the DGP_RF constructor arguments,
 * models/dgp.py:9-52 + the minibatch size and chain count); dgprf_plan_init derives the rest:
 * per-layer widths (models/dgp.py:74-91), Phi widths (models/dgp.py:103,107), the packed
 * parameter layout in HBM and the step-kernel workspace.
 *
 * Packed HBM layouts (floats):
 *   theta / momenta [n_chains][w_total]  : W_l [P_l][g_l] at w_off[l]    (GPLayer.W, dgp.py:66-68)
 *   z / omega       [omega_total]        : [d_l][R_l] at omega_off[l]    (RBFLayer.z / Omega)
 *   hyp             [hyp_total]          : log_amp[L], lik_log_var, pad, log_inv_ls (sum d_l) at
 *                                          lis_off[l], mean (sum d_l) at mean_off[l]
 *   der             [der_total]          : c_l = amp/sqrt(R) (RBF) or sqrt2*amp/sqrt(R) (ARC),
 *                                          then sigma^2 at der[DGPRF_MAX_LAYERS]
 *   mass            [n_chains][n_layers] : preconditioner M per W_l (models/dgp.py:235-237)
 *   workspace       [ws_total]           : step-kernel partials (per chain ws_chain floats); zero-fill
 *                                          it once before first use (it holds the full-Bayes
 *                                          arrival counters, which the kernels leave at zero)
 */
typedef struct dgprf_plan {
  /* ---- caller ---- */
  int32_t n_layers;
  int32_t d_in;
  int32_t d_out;
  int32_t input_cat;
  int32_t likelihood;
  int32_t batch;        /* minibatch rows B the step kernels are sized for */
  int32_t n_chains;     /* independent chains sharing Omega (one posterior) */
  int32_t kind[DGPRF_MAX_LAYERS];
  int32_t n_rf[DGPRF_MAX_LAYERS];
  int32_t n_gp[DGPRF_MAX_LAYERS];
  int32_t hyp_flags;       /* DGPRF_HYP_* groups that are trainable (full_bayesian=True) */
  int32_t hyp_per_chain;   /* 1: hyp / omega / der are per chain ([C][...]); 0: shared */
  int32_t ard[DGPRF_MAX_LAYERS]; /* 1: per-dimension log_inv_ls; 0: one scalar (d equal slots) */
  int32_t fwd_path;        /* DGPRF_FWD_* (0 = AUTO) */
  int32_t agemm_chunk_rows; /* wide first layer: rows of A_1 per dgprf_forward chunk (0 = as many as
                               fit 64M floats; otherwise rounded down to a multiple of 64, >= 64) */
  int32_t fresh_z;         /* bit l: layer l draws fresh z ~ N(0,1) every step (random_fixed=False,
                              layers/rf_layers.py:39-41): the step builds that layer's Omega from
                              Philox (seed, sub = step, DGPRF_RNG_Z, tag = 1 + l + 16 chain) into
                              the workspace (omf_off).  W-only steps (not full_bayes). */
  int32_t bwd_tiles;       /* 1: keep the per-row-tile backward (one gW partial row per 16-row tile)
                              whatever B.  For full_bayesian=True steps / gradients at B > 256 when
                              some layer does not fit the full-Bayes row-group layout
                              (rg_full_bayes == 0, e.g. BASELINE config 4's 784-wide layer); ABI 7 */
  /* ---- derived by dgprf_plan_init ---- */
  int32_t initialised;
  int32_t d[DGPRF_MAX_LAYERS];      /* layer input width */
  int32_t P[DGPRF_MAX_LAYERS];      /* Phi width: 2R (RBF) or R (ARC) */
  int32_t ns[DGPRF_MAX_LAYERS];     /* feature slices per step kernel */
  int32_t cpw[DGPRF_MAX_LAYERS];    /* 16-feature chunks per wave per slice */
  int32_t n_row_tiles;              /* ceil(B/16) */
  int32_t n_rt_pad;                 /* n_gw_rows rounded up to 16 (zero rows in gW partials) */
  int32_t rt_per_group;             /* row tiles per backward workgroup: 1 while B <= 256 (one gW
                                       partial row per row tile), ceil(n_row_tiles / 16) beyond, so
                                       the gW partials stay <= 16 rows whatever B (row-group
                                       backward; 1 also when some layer does not fit it)        */
  int32_t n_gw_rows;                /* gW partial rows: ceil(n_row_tiles / rt_per_group) <= 16
                                       (or n_row_tiles when rt_per_group == 1)                  */
  int32_t rg_full_bayes;            /* rt_per_group > 1: every layer also fits the full-Bayes
                                       row-group backward (else full_bayes steps / gradients
                                       return DGPRF_E_SHAPE for this batch size)                */
  int32_t fold_out;                 /* 1: W-only steps fold the output layer's forward into its
                                       backward — every backward workgroup of layer L recomputes
                                       its 16 rows of F_L over all R_L features instead of summing
                                       the 16 slice partials of a separate forward launch (one
                                       launch and one dependent boundary fewer per step; g_L = 1
                                       Gaussian output layers with a small d_L R_L, B <= 256,
                                       fewer than 4 chains); ABI 10 */
  int64_t omega_off[DGPRF_MAX_LAYERS];
  int64_t w_off[DGPRF_MAX_LAYERS];
  int64_t lis_off[DGPRF_MAX_LAYERS];
  int64_t mean_off[DGPRF_MAX_LAYERS];
  int64_t fp_off[DGPRF_MAX_LAYERS];  /* F partials  [16][B][g] (per chain; slices >= ns stay 0) */
  int64_t dxp_off[DGPRF_MAX_LAYERS]; /* dX partials [16][B][g_{l-1}] (per chain, l>=1)      */
  int64_t gwp_off;                   /* gW partials [n_rt_pad][w_total] (per chain; rows past
                                        n_gw_rows stay zero)                                    */
  int64_t logp_off;                  /* per-row minibatch log p [B] (per chain) */
  int64_t omega_total;
  int64_t w_total;
  int64_t hyp_total;
  int64_t der_total;
  int64_t ws_chain;
  int64_t ws_total;
  int64_t hpp_off[DGPRF_MAX_LAYERS]; /* full-Bayes partials [n_rt_pad][16][align4(2 d_l + 1)] (per chain) */
  int64_t hpl_off;                   /* full-Bayes lik_log_var partials [n_rt_pad], then 8 uint32
                                        arrival counters of the hyper workgroups (per chain)
                                        and the eager step-advance counter (chain 0)          */
  int64_t xb_off;                    /* gathered minibatch rows X [B][d_in] (per chain)        */
  int64_t yb_off;                    /* gathered minibatch targets [B][yb_cols] (per chain)    */
  int32_t yb_cols;                   /* g_L (Gaussian) or 1 (softmax label)                    */
  int32_t pad0;
  int64_t a0_off;                    /* layer 1 with d > 32 (e.g. the 784-wide MNIST input):
                                        A_1 = X Omega_1 [align32(B)][R_1] precomputed by one tiled
                                        MFMA GEMM per step (per chain); -1 when not used          */
  int64_t omf_off;                   /* fresh_z != 0: this step's Omega of every layer [omega_total]
                                        (per chain; fresh layers rebuilt each step); -1 otherwise */
} dgprf_plan_t;

/* Device state of the chains.  Replaces the tf.Variables W and their ad-hoc attributes
 * `moments` and `M` (models/dgp.py:208-216, 235-240). */
typedef struct dgprf_chain {
  float *theta;          /* [C][w_total] */
  float *mom;            /* [C][w_total] */
  float *omega;          /* [omega_total] or [C][omega_total] (from dgprf_omega_build) */
  float *der;            /* [der_total] or [C][der_total]     (from dgprf_omega_build) */
  const float *mass;     /* [C][n_layers] */
  /* full_bayesian=True state (may be NULL otherwise): */
  const float *z;        /* [omega_total] RF base frequencies (Omega is rebuilt after updates) */
  float *hyp;            /* [hyp_total] or [C][hyp_total] */
  float *hmom;           /* [C][hyp_total] hyper-parameter momenta (hyp layout) */
  const float *hmass;    /* [C][DGPRF_HMASS] */
  float *ws;             /* [ws_total] */
  int64_t *step;         /* device step counter (Philox counter / minibatch position) */
  uint64_t seed;         /* Philox key (already folded with the rank by the host) */
} dgprf_chain_t;

/* Minibatch source (replaces the host tf.data iterator, experiments/utils_dataset.py:26-44). */
typedef struct dgprf_batch {
  const float *X;        /* [n_data][d_in] */
  const float *Y;        /* [n_data][y_cols] (softmax: class label as float in column 0) */
  const int32_t *idx;    /* DGPRF_BATCH_INDEXED: [C][B] */
  int64_t n_data;
  int32_t y_cols;
  int32_t mode;
  int64_t iters_per_epoch;  /* DGPRF_BATCH_EPOCH: floor(n_data / B) */
  uint64_t perm_seed;       /* DGPRF_BATCH_EPOCH */
  const float *A1;          /* optional, wide first layer (plan.a0_off >= 0): X Omega_1 of every
                               dataset row [n_data][n_rf[0]] (dgprf_rf_project of the whole
                               dataset, kept resident in HBM).  W-only steps of an EPOCH / INDEXED
                               batch then gather their minibatch's rows of it instead of running
                               the A_1 GEMM every step (Omega_1 is fixed unless full_bayes or layer
                               0 draws fresh z; both ignore A1).  The caller recomputes it whenever
                               Omega_1 changes.  NULL: the GEMM.  ABI 8 */
} dgprf_batch_t;

/* One SGHMC/SGLD update's scalars: DGP_RF.sgmcmc_update(..., data_size, lr, momentum_decay,
 * resample_moments, temperature) (models/dgp.py:184-216). */
typedef struct dgprf_step {
  float lr;
  float momentum_decay;
  float temperature;
  float data_size;          /* N */
  int32_t resample_moments;
  int32_t schedule;         /* DGPRF_SCHED_* */
  int32_t step_offset;      /* added to *chain.step (graph sub-step index) */
  int32_t grad_only;        /* internal: set by dgprf_potential_grad */
  /* DGPRF_SCHED_CYCLICAL (experiments/utils_training.py:47-61): */
  int64_t start_step;       /* first sampling step (start_sampling_epoch * iters) */
  int64_t cycle_length;     /* epochs_per_cycle * iters */
  int32_t resample_in_cycle_head;
  int32_t full_bayes;       /* full_bayesian=True: also update the plan.hyp_flags groups */
  /* optional injected standard normals (parity tests; NULL = device Philox): */
  const float *xi;          /* [C][w_total] noise */
  const float *xi_resample; /* [C][w_total] resampled momenta */
  const float *xi_hyp;          /* [C][hyp_total] hyper-parameter noise (hyp layout) */
  const float *xi_hyp_resample; /* [C][hyp_total] resampled hyper-parameter momenta */
} dgprf_step_t;

typedef struct dgprf_graph *dgprf_graph_handle;

/* ---------------- meta ---------------- */
int dgprf_abi_version(void);
const char *dgprf_error_string(int code);
/* Derive the plan (models/dgp.py:34-115).  Host-only, no device work. */
int dgprf_plan_init(dgprf_plan_t *plan);

/* ---------------- initial draws ---------------- */
/* Fill out[n] with N(0,1) from Philox4x32-10 (key = seed, counter = (i/4, sub_lo, sub_hi,
 * purpose<<24)) + Box-Muller.  Replaces tf.random.normal at layers/rf_layers.py:22,
 * layers/GP_weight_layers.py:9, models/dgp.py:210,212,240. */
int dgprf_philox_normal(float *out, int64_t n, uint64_t seed, uint64_t subsequence,
                        uint32_t purpose, void *stream);

/* ---------------- kernel hyper-parameters ---------------- */
/* Omega_l = exp(log_inv_ls_l)[:,None] * z_l + mean_l, c_l and sigma^2 into der.
 * Replaces kernels/RBF.py:43-53, kernels/arc_cosine.py:46-56, layers/rf_layers.py:34-38,44,90,
 * likelihoods/gaussian.py:14-16. */
int dgprf_omega_build(const dgprf_plan_t *plan, const float *z, const float *hyp, float *omega,
                      float *der, void *stream);  /* hyp_per_chain: every chain's [C][...] */

/* ---------------- the hot path ---------------- */
/* One full SGHMC/SGLD step for every chain: minibatch gather, forward through all L layers
 * (Omega x -> cos|sin or relu -> Phi W), likelihood, analytic backward (gW_l = Phi_l^T dF_l +
 * W_l/N), and the fused update with device Philox noise.  Advances *chain.step by one.
 * Replaces DGP_RF.sgmcmc_update (models/dgp.py:184-216); step.full_bayes = full_bayesian=True:
 * the plan.hyp_flags hyper-parameters take the same update from their gradients (needs chain.z,
 * hyp, hmom, hmass) and Omega / c / sigma^2 are rebuilt after it. */
int dgprf_sghmc_step(const dgprf_plan_t *plan, const dgprf_chain_t *chain,
                     const dgprf_batch_t *batch, const dgprf_step_t *step, void *stream);

/* Gradient of U w.r.t. every W_l (models/dgp.py:161-182 + tape.gradient :194-198) into
 * grad_out [C][w_total]; full_bayes: w.r.t. every trainable variable (:175-181, 199-204) into
 * grad_out [C][w_total + hyp_total] (hyper-parameter gradients in the hyp layout; a scalar
 * length scale's gradient is written to all d of its slots; slots of groups that do not train
 * and padding slots are 0).  No update, step counter untouched. */
int dgprf_potential_grad(const dgprf_plan_t *plan, const dgprf_chain_t *chain,
                         const dgprf_batch_t *batch, float data_size, int32_t full_bayes,
                         float *grad_out, void *stream);

/* Capture `steps_per_graph` consecutive dgprf_sghmc_step calls (sub-step k uses
 * step_offset = k, then *step += steps_per_graph) into one hipGraph. */
int dgprf_graph_create_sghmc(dgprf_graph_handle *out, const dgprf_plan_t *plan,
                             const dgprf_chain_t *chain, const dgprf_batch_t *batch,
                             const dgprf_step_t *step, int32_t steps_per_graph);
int dgprf_graph_launch(dgprf_graph_handle graph, void *stream);
int dgprf_graph_destroy(dgprf_graph_handle graph);

/* Per-kernel device time of the step sequence, measured with hipEvents on `stream`: `reps` real
 * steps (forward l = 0..L-1, backward L-1..0, update; the chain advances) with an event pair around
 * every kernel.  ms_out[k] (2L + 3 entries) receives the mean milliseconds of the pair around kernel
 * k, indexed forward l -> l, backward l -> L + l, update -> 2L, ms_out[2L + 1] the mean of an
 * empty pair recorded the same way (the pair's own cost, to subtract), and ms_out[2L + 2] the pair
 * around the A_1 = X Omega_1 GEMM of a wide first layer (0 without one; forward 0 then excludes
 * it).  ABI 6: the A_1 slot. */
int dgprf_profile_step(const dgprf_plan_t *plan, const dgprf_chain_t *chain,
                       const dgprf_batch_t *batch, const dgprf_step_t *step, int32_t reps,
                       float *ms_out, void *stream);

/* ---------------- predictive / forward ---------------- */
/* Floats of device scratch dgprf_forward needs for n rows (0 unless the first layer is wide and the
 * A_1 GEMM path is taken).  Host-only. */
int dgprf_forward_scratch(const dgprf_plan_t *plan, int64_t n, int64_t *floats_out);

/* Forward of n rows through all layers for every chain (BNN_from_list.__call__, utils.py:10-16;
 * BNN_from_list_input_cat.__call__, utils.py:32-44) plus the likelihood
 * (RegressionDGP.eval_log_likelihood_and_se, models/regression_model.py:33-50;
 * ClassificationDGP.eval_log_likelihood, models/classification_model.py:49-60).
 * Optional outputs (NULL to skip), each with a per-chain stride of n rows:
 *   f_out[l]  [C][n][g_l]   per-layer outputs (feed_forward_all_layers, regression_model.py:24-31)
 *   logp      [C][n]        log p(y|F)
 *   se        [C][n]        mean_k (y - f)^2 (Gaussian only)
 *   lse_m/lse_s/se_sum [C][n]  online log-sum-exp over samples (experiments/utils_training.py:79-85)
 *                         updated in place: m' = max(m, lp); s' = s e^{m-m'} + e^{lp-m'}.
 * Y may be NULL when no likelihood output is requested.  omega/der are [C][...] when
 * plan.hyp_per_chain (chain c scored with its own hyper-parameters).  scratch: >= the floats
 * dgprf_forward_scratch reports for n (may be NULL when that is 0); owned by the caller. */
int dgprf_forward(const dgprf_plan_t *plan, const float *theta, const float *omega,
                  const float *der, const float *X, const float *Y, int32_t y_cols, int64_t n,
                  float *const *f_out, float *logp, float *se, float *lse_m, float *lse_s,
                  float *se_sum, float *scratch, int64_t scratch_floats, void *stream);

/* Posterior-predictive fold of several posterior samples of every chain (the driver's loop over W
 * samples, experiments/utils_training.py:79-85): thetas [n_samples][n_chains][w_total]; each
 * sample's per-row log p (and squared error) is folded into the chain's online log-sum-exp
 * accumulators lse_m / lse_s (and se_sum, Gaussian) [n_chains][n] in sample order, as n_samples
 * dgprf_forward calls would (the same bits).  Lean models (every layer d, g <= 8, n large enough
 * for the tile kernel) score two samples per pass with layer 0 computed once for the pair (Omega
 * is fixed across samples, layers/rf_layers.py:21-22); other models run the one-sample kernels.
 * With scratch_floats >= dgprf_forward_samples_scratch every sample (pair) runs in ONE launch and
 * scratch receives the per-row log p / squared errors [n_samples][n_chains][n] that a fold kernel
 * then applies in sample order; with less, one launch per sample (pair) folds in place.  ABI 8;
 * the one-launch form ABI 9. */
/* Floats of device scratch that let dgprf_forward_samples score n_samples samples of n rows in its
 * fastest form (every sample pair in one launch, then a fold in sample order; at least the
 * dgprf_forward_scratch figure).  Less scratch still works: one launch per pair.  Host-only.  ABI 9. */
int dgprf_forward_samples_scratch(const dgprf_plan_t *plan, int64_t n, int32_t n_samples,
                                  int64_t *floats_out);
int dgprf_forward_samples(const dgprf_plan_t *plan, const float *thetas, int32_t n_samples,
                          const float *omega, const float *der, const float *X, const float *A1,
                          const float *Y, int32_t y_cols, int64_t n, float *lse_m, float *lse_s,
                          float *se_sum, float *scratch, int64_t scratch_floats, void *stream);
/* (A1: optional [align64(n)][n_rf[0]] = X Omega_1 for a wide first layer (plan.a0_off >= 0),
 * computed once by dgprf_rf_project and shared by every sample — Omega_1 is fixed across samples
 * — so no sample runs the A_1 GEMM; rows n .. align64(n) are read (whole 64-row workgroups) and
 * their outputs discarded.  NULL: the GEMM per sample, in scratch chunks.) */
/* Posterior-predictive summary (experiments/utils_training.py:79-85):
 * per point lse[n] = log sum_s exp(lp_s) over all chains' accumulators, and
 * out[0] = mean_n(lse - log S_total) - log_y_std, out[1] = sqrt(sum se / (S_total n)) * y_std.
 * lse_m/lse_s/se_sum are [parts][n] (chains x ranks), combined in fixed order. */
int dgprf_lse_finalize(const float *lse_m, const float *lse_s, const float *se_sum,
                       int32_t parts, int64_t n, double s_total, float log_y_std, float y_std,
                       float *lse_out, double *out, void *stream);

/* Omega and c of ONE stand-alone RF layer (RBFLayer / ARCLayer outside a DGP_RF):
 * omega[d][R] = exp(log_inv_ls)[:,None] z + mean[:,None]; c[0] = amp/sqrt(R) or sqrt2 amp/sqrt(R).
 * layers/rf_layers.py:34-44, 80-90; kernels/RBF.py:43-53. */
int dgprf_rf_omega(int32_t kind, int32_t d, int32_t R, const float *z, const float *log_inv_ls,
                   const float *mean, const float *log_amp, float *omega, float *c, void *stream);

/* Single RF layer features (RBFLayer.__call__ layers/rf_layers.py:29-45, ARCLayer.__call__
 * :75-91): phi[n][P] = c * [cos(XOmega) | sin(XOmega)] or c * relu(XOmega). */
int dgprf_rf_features(int32_t kind, const float *X, int64_t n, int32_t d, const float *omega,
                      int32_t R, const float *c, float *phi, void *stream);
/* GPLayer.__call__ (layers/GP_weight_layers.py:11-15): F[n][g] = Phi[n][P] W[P][g]. */
int dgprf_gp_matmul(const float *phi, int64_t n, int32_t P, const float *W, int32_t g, float *F,
                    void *stream);
/* The RF projection of one layer, A = X Omega (RBFLayer / ARCLayer `tf.matmul(x, self.Omega)`,
 * layers/rf_layers.py:42, 88): A[n][R] = X[n][0:d] Omega[d][R], X with row stride ldx >= d, as the
 * hand-written fp32 MFMA GEMM the wide first layer of the step and of the predictive forward runs
 * (64 x 64 tiles with K whole up to 1,024 rows, 128 x 128 beyond; the step's own A_1 GEMM runs
 * 64 x 64 tiles in two K parts).  d, ldx and R multiples of 4 for the MFMA
 * kernel (other shapes take the LDS-tiled 16x16x4 fallback).  ABI 7. */
int dgprf_rf_project(const float *X, int64_t n, int32_t ldx, int32_t d, const float *omega,
                     int32_t R, float *A, void *stream);

/* sum log N(W;0,1) per chain (DGP_RF.prior_W, models/dgp.py:129-136) into out[C]. */
int dgprf_prior_w(const dgprf_plan_t *plan, const float *theta, float *out, void *stream);

/* ---------------- update / preconditioner ---------------- */
/* Stand-alone SGHMC update of theta/mom from a given gradient grad [C][w_total]
 * (models/dgp.py:206-216).  Uses *step + step->step_offset for the Philox counter. */
int dgprf_sghmc_update(const dgprf_plan_t *plan, float *theta, float *mom, const float *grad,
                       const float *mass, const int64_t *step_ctr, uint64_t seed,
                       const dgprf_step_t *step, void *stream);
/* Welford accumulation of one gradient sample (models/dgp.py:259-271):
 * k is the 1-based sample index; grad/mean/m2 [C][w_total] (full_bayes: [C][w_total + hyp_total]). */
int dgprf_welford_update(const dgprf_plan_t *plan, const float *grad, float *mean, float *m2,
                         int32_t k, int32_t full_bayes, void *stream);
/* Mass estimate per variable (models/dgp.py:276-288): W_l into mass_est [C][L]; full_bayes: also
 * the trainable hyper-parameter variables into hmass_est [C][DGPRF_HMASS] (other slots 0).
 * centered: sqrt(mean(m2/(K-1)) + 1e-7); else sqrt(mean(mean^2 + m2/K) + 1e-7). */
int dgprf_mass_estimate(const dgprf_plan_t *plan, const float *mean, const float *m2,
                        int32_t k_batches, int32_t centered, int32_t full_bayes, float *mass_est,
                        float *hmass_est, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* DGPRF_H */
