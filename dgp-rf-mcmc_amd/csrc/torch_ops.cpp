// torch_ops.cpp — the hot-path entry points of libdgprf.so registered as PyTorch operators
// (TORCH_LIBRARY(dgprf, m)), so torch's dispatcher, its current HIP stream and torch.cuda.graph
// capture see the work.  Each op validates its tensors (device, dtype, contiguity, sizes against the
// plan), assembles the C-ABI structs of include/dgprf.h and calls the extern "C" entry point on the
// current HIP stream.  The plan travels as a CPU uint8 tensor holding a dgprf_plan_t filled by
// dgprf_plan_init (dgprf/_native.py make_plan), i.e. the model shape of DGP_RF.__init__
// (models/dgp.py:9-115).
//
//   dgprf::sghmc_step_     DGP_RF.sgmcmc_update            models/dgp.py:184-216
//   dgprf::potential_grad  U + tape.gradient               models/dgp.py:161-182, 194-204
//   dgprf::forward         BNN(X) + eval_log_likelihood(_and_se) + online LSE fold
//                          utils.py:10-44, models/regression_model.py:33-50,
//                          experiments/utils_training.py:63-65
//   dgprf::lse_finalize    experiments/utils_training.py:79-85
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include <ATen/ops/empty.h>
#include <ATen/ops/zeros.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include "../../include/dgprf.h"

namespace {

using at::Tensor;
using OptT = std::optional<Tensor>;

void check_rc(int rc, const char* fn) {
  if (rc == DGPRF_OK) return;
  if (rc == DGPRF_E_SHAPE) TORCH_CHECK_VALUE(false, fn, ": unsupported shape (", dgprf_error_string(rc), ")");
  TORCH_CHECK(false, fn, " failed: ", dgprf_error_string(rc), " (code ", rc, ")");
}

dgprf_plan_t plan_of(const Tensor& p) {
  TORCH_CHECK(p.device().is_cpu() && p.scalar_type() == at::kByte && p.is_contiguous() &&
                  p.numel() == (int64_t)sizeof(dgprf_plan_t),
              "dgprf: plan must be a CPU uint8 tensor of sizeof(dgprf_plan_t) bytes");
  dgprf_plan_t pl;
  std::memcpy(&pl, p.data_ptr(), sizeof(pl));
  TORCH_CHECK(pl.initialised == 1, "dgprf: plan not initialised (dgprf_plan_init)");
  return pl;
}

void* stream() { return c10::hip::getCurrentHIPStream().stream(); }

// device fp32 contiguous with at least `n` elements (n < 0: any size)
float* f32(const Tensor& t, const char* what, int64_t n = -1) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous(), "dgprf: ", what,
              " must be a contiguous float32 HIP tensor");
  TORCH_CHECK(n < 0 || t.numel() >= n, "dgprf: ", what, " has ", t.numel(), " elements, needs ", n);
  return t.data_ptr<float>();
}
float* f32o(const OptT& t, const char* what, int64_t n = -1) {
  return t.has_value() && t->defined() ? f32(*t, what, n) : nullptr;
}

dgprf_batch_t batch_of(const dgprf_plan_t& pl, const Tensor& X, const Tensor& Y, int64_t mode,
                       int64_t iters, int64_t perm_seed, const OptT& idx) {
  TORCH_CHECK(X.dim() == 2 && X.size(1) == pl.d_in, "dgprf: X must be [n, d_in]");
  TORCH_CHECK(Y.dim() == 2 && Y.size(0) == X.size(0), "dgprf: Y must be [n, y_cols]");
  dgprf_batch_t b;
  std::memset(&b, 0, sizeof(b));  // A1 = NULL: eager calls run the A_1 GEMM
  b.X = f32(X, "X");
  b.Y = f32(Y, "Y");
  b.n_data = X.size(0);
  b.y_cols = (int32_t)Y.size(1);
  b.mode = (int32_t)mode;
  b.iters_per_epoch = iters;
  b.perm_seed = (uint64_t)perm_seed;
  if (idx.has_value() && idx->defined()) {
    TORCH_CHECK(idx->is_cuda() && idx->scalar_type() == at::kInt && idx->is_contiguous() &&
                    idx->numel() >= (int64_t)pl.n_chains * pl.batch,
                "dgprf: idx must be int32 [C, B] on the device");
    b.idx = idx->data_ptr<int32_t>();
  }
  return b;
}

dgprf_chain_t chain_of(const dgprf_plan_t& pl, const Tensor& theta, const Tensor& mom,
                       const Tensor& omega, const Tensor& der, const Tensor& mass,
                       const Tensor& ws, const Tensor& step, int64_t seed, const OptT& z,
                       const OptT& hyp, const OptT& hmom, const OptT& hmass) {
  const int64_t C = pl.n_chains, ch = pl.hyp_per_chain ? C : 1;
  dgprf_chain_t c;
  std::memset(&c, 0, sizeof(c));
  c.theta = f32(theta, "theta", C * pl.w_total);
  c.mom = f32(mom, "mom", C * pl.w_total);
  c.omega = f32(omega, "omega", ch * pl.omega_total);
  c.der = f32(der, "der", ch * pl.der_total);
  c.mass = f32(mass, "mass", C * pl.n_layers);
  c.ws = f32(ws, "ws", pl.ws_total);
  TORCH_CHECK(step.is_cuda() && step.scalar_type() == at::kLong && step.numel() >= 1,
              "dgprf: step must be an int64 HIP tensor");
  c.step = step.data_ptr<int64_t>();
  c.seed = (uint64_t)seed;
  c.z = f32o(z, "z", pl.omega_total);
  c.hyp = f32o(hyp, "hyp", ch * pl.hyp_total);
  c.hmom = f32o(hmom, "hmom", C * pl.hyp_total);
  c.hmass = f32o(hmass, "hmass", C * DGPRF_HMASS);
  return c;
}

void sghmc_step_(const Tensor& plan, const Tensor& theta, const Tensor& mom, const Tensor& omega,
                 const Tensor& der, const Tensor& mass, const Tensor& ws, const Tensor& step,
                 int64_t seed, const Tensor& X, const Tensor& Y, int64_t mode, int64_t iters,
                 int64_t perm_seed, const OptT& idx, double lr, double momentum_decay,
                 double temperature, double data_size, bool resample, const OptT& xi,
                 const OptT& xi_resample, bool full_bayes, const OptT& z, const OptT& hyp,
                 const OptT& hmom, const OptT& hmass, const OptT& xi_hyp,
                 const OptT& xi_hyp_resample) {
  const dgprf_plan_t pl = plan_of(plan);
  const dgprf_chain_t c = chain_of(pl, theta, mom, omega, der, mass, ws, step, seed, z, hyp, hmom, hmass);
  const dgprf_batch_t b = batch_of(pl, X, Y, mode, iters, perm_seed, idx);
  dgprf_step_t st;
  std::memset(&st, 0, sizeof(st));
  st.lr = (float)lr;
  st.momentum_decay = (float)momentum_decay;
  st.temperature = (float)temperature;
  st.data_size = (float)data_size;
  st.resample_moments = resample ? 1 : 0;
  st.schedule = DGPRF_SCHED_CONST;
  st.cycle_length = 1;
  st.full_bayes = full_bayes ? 1 : 0;
  const int64_t nw = (int64_t)pl.n_chains * pl.w_total, nh = (int64_t)pl.n_chains * pl.hyp_total;
  st.xi = f32o(xi, "xi", nw);
  st.xi_resample = f32o(xi_resample, "xi_resample", nw);
  st.xi_hyp = f32o(xi_hyp, "xi_hyp", nh);
  st.xi_hyp_resample = f32o(xi_hyp_resample, "xi_hyp_resample", nh);
  check_rc(dgprf_sghmc_step(&pl, &c, &b, &st, stream()), "dgprf_sghmc_step");
}

Tensor potential_grad(const Tensor& plan, const Tensor& theta, const Tensor& omega,
                      const Tensor& der, const Tensor& mass, const Tensor& ws, const Tensor& step,
                      const Tensor& X, const Tensor& Y, int64_t mode, int64_t iters,
                      int64_t perm_seed, const OptT& idx, double data_size, bool full_bayes,
                      const OptT& z, const OptT& hyp, const OptT& hmom, const OptT& hmass) {
  const dgprf_plan_t pl = plan_of(plan);
  // the gradient pass reads but never writes theta / mom (mom only by the update)
  const dgprf_chain_t c = chain_of(pl, theta, theta, omega, der, mass, ws, step, 0, z, hyp, hmom, hmass);
  const dgprf_batch_t b = batch_of(pl, X, Y, mode, iters, perm_seed, idx);
  const int64_t n = pl.w_total + (full_bayes ? pl.hyp_total : 0);
  Tensor out = at::empty({(int64_t)pl.n_chains, n}, theta.options());
  check_rc(dgprf_potential_grad(&pl, &c, &b, (float)data_size, full_bayes ? 1 : 0,
                                out.data_ptr<float>(), stream()),
           "dgprf_potential_grad");
  return out;
}

std::tuple<std::vector<Tensor>, Tensor, Tensor> forward(
    const Tensor& plan, const Tensor& theta, const Tensor& omega, const Tensor& der,
    const Tensor& X, const OptT& Y, int64_t f_mask, bool logp, bool se, const OptT& lse_m,
    const OptT& lse_s, const OptT& se_sum, const OptT& scratch) {
  const dgprf_plan_t pl = plan_of(plan);
  const int64_t C = pl.n_chains, ch = pl.hyp_per_chain ? C : 1;
  TORCH_CHECK(X.dim() == 2 && X.size(1) == pl.d_in, "dgprf: X must be [n, d_in]");
  const int64_t n = X.size(0);
  float* Yp = nullptr;
  int32_t y_cols = 0;
  if (Y.has_value() && Y->defined()) {
    TORCH_CHECK(Y->dim() == 2 && Y->size(0) == n, "dgprf: Y must be [n, y_cols]");
    Yp = f32(*Y, "Y");
    y_cols = (int32_t)Y->size(1);
  }
  std::vector<Tensor> F;
  float* fptr[DGPRF_MAX_LAYERS] = {};
  for (int l = 0; l < pl.n_layers; ++l)
    if (f_mask & (1ll << l)) {
      F.push_back(at::empty({C, n, (int64_t)pl.n_gp[l]}, theta.options()));
      fptr[l] = F.back().data_ptr<float>();
    }
  Tensor lp = logp ? at::empty({C, n}, theta.options()) : at::empty({0}, theta.options());
  Tensor sq = se ? at::empty({C, n}, theta.options()) : at::empty({0}, theta.options());
  int64_t need = 0;
  check_rc(dgprf_forward_scratch(&pl, n, &need), "dgprf_forward_scratch");
  float* scr = f32o(scratch, "scratch", need);
  TORCH_CHECK(need == 0 || scr, "dgprf: forward needs ", need, " floats of scratch");
  check_rc(dgprf_forward(&pl, f32(theta, "theta", C * pl.w_total), f32(omega, "omega", ch * pl.omega_total),
                         f32(der, "der", ch * pl.der_total), f32(X, "X"), Yp, y_cols, n, fptr,
                         logp ? lp.data_ptr<float>() : nullptr, se ? sq.data_ptr<float>() : nullptr,
                         f32o(lse_m, "lse_m", C * n), f32o(lse_s, "lse_s", C * n),
                         f32o(se_sum, "se_sum", C * n), scr,
                         scr ? scratch->numel() : 0, stream()),
           "dgprf_forward");
  return {F, lp, sq};
}

// thetas [S][C][w_total]: every sample of every chain folded into the LSE accumulators [C][n]
void forward_samples(const Tensor& plan, const Tensor& thetas, const Tensor& omega,
                     const Tensor& der, const Tensor& X, const OptT& A1, const Tensor& Y,
                     const Tensor& lse_m, const Tensor& lse_s, const OptT& se_sum,
                     const OptT& scratch) {
  const dgprf_plan_t pl = plan_of(plan);
  const int64_t C = pl.n_chains, ch = pl.hyp_per_chain ? C : 1;
  TORCH_CHECK(X.dim() == 2 && X.size(1) == pl.d_in, "dgprf: X must be [n, d_in]");
  const int64_t n = X.size(0);
  TORCH_CHECK(Y.dim() == 2 && Y.size(0) == n, "dgprf: Y must be [n, y_cols]");
  TORCH_CHECK(thetas.dim() == 3 && thetas.size(1) == C && thetas.size(2) == pl.w_total,
              "dgprf: thetas must be [samples, n_chains, w_total]");
  const int64_t S = thetas.size(0);
  // A1 rows past n up to a multiple of 64 are read (whole 64-row tile-kernel workgroups)
  float* a1 = f32o(A1, "A1", (n + 63) / 64 * 64 * (int64_t)pl.n_rf[0]);
  int64_t need = 0;
  check_rc(dgprf_forward_scratch(&pl, n, &need), "dgprf_forward_scratch");
  // the A_1 chunks need `need` floats unless A1 is resident; more (dgprf_forward_samples_scratch)
  // lets every sample pair run in one launch
  float* scr = f32o(scratch, "scratch", a1 ? 0 : need);
  TORCH_CHECK(a1 || need == 0 || scr, "dgprf: forward needs ", need, " floats of scratch");
  check_rc(dgprf_forward_samples(&pl, f32(thetas, "thetas", S * C * pl.w_total), (int32_t)S,
                                 f32(omega, "omega", ch * pl.omega_total),
                                 f32(der, "der", ch * pl.der_total), f32(X, "X"), a1, f32(Y, "Y"),
                                 (int32_t)Y.size(1), n, f32(lse_m, "lse_m", C * n),
                                 f32(lse_s, "lse_s", C * n), f32o(se_sum, "se_sum", C * n), scr,
                                 scr ? scratch->numel() : 0, stream()),
           "dgprf_forward_samples");
}

std::tuple<Tensor, Tensor> lse_finalize(const Tensor& m, const Tensor& s, const OptT& e,
                                        double s_total, double y_std, bool lse_out) {
  TORCH_CHECK(m.dim() == 2 && s.sizes() == m.sizes(), "dgprf: accumulators must be [parts, n]");
  const int64_t parts = m.size(0), n = m.size(1);
  Tensor out = at::zeros({2}, m.options().dtype(at::kDouble));
  Tensor lo = lse_out ? at::empty({n}, m.options()) : at::empty({0}, m.options());
  check_rc(dgprf_lse_finalize(f32(m, "lse_m", parts * n), f32(s, "lse_s", parts * n),
                              f32o(e, "se_sum", parts * n), (int32_t)parts, n, s_total,
                              (float)std::log(y_std), (float)y_std,
                              lse_out ? lo.data_ptr<float>() : nullptr, out.data_ptr<double>(),
                              stream()),
           "dgprf_lse_finalize");
  return {out, lo};
}

}  // namespace

TORCH_LIBRARY(dgprf, m) {
  m.def(
      "sghmc_step_(Tensor plan, Tensor(a!) theta, Tensor(b!) mom, Tensor(c!) omega, Tensor(d!) der, "
      "Tensor mass, Tensor(e!) ws, Tensor(f!) step, int seed, Tensor X, Tensor Y, int mode, "
      "int iters_per_epoch, int perm_seed, Tensor? idx, float lr, float momentum_decay, "
      "float temperature, float data_size, bool resample_moments, Tensor? xi, Tensor? xi_resample, "
      "bool full_bayes, Tensor? z, Tensor(g!)? hyp, Tensor(h!)? hmom, Tensor? hmass, "
      "Tensor? xi_hyp, Tensor? xi_hyp_resample) -> ()");
  m.def(
      "potential_grad(Tensor plan, Tensor theta, Tensor omega, Tensor der, Tensor mass, "
      "Tensor(a!) ws, Tensor step, Tensor X, Tensor Y, int mode, int iters_per_epoch, "
      "int perm_seed, Tensor? idx, float data_size, bool full_bayes, Tensor? z, Tensor? hyp, "
      "Tensor? hmom, Tensor? hmass) -> Tensor");
  m.def(
      "forward(Tensor plan, Tensor theta, Tensor omega, Tensor der, Tensor X, Tensor? Y, "
      "int f_mask, bool logp, bool se, Tensor(a!)? lse_m, Tensor(b!)? lse_s, Tensor(c!)? se_sum, "
      "Tensor(d!)? scratch) -> (Tensor[], Tensor, Tensor)");
  m.def(
      "forward_samples(Tensor plan, Tensor thetas, Tensor omega, Tensor der, Tensor X, Tensor? A1, "
      "Tensor Y, Tensor(a!) lse_m, Tensor(b!) lse_s, Tensor(c!)? se_sum, Tensor(d!)? scratch) "
      "-> ()");
  m.def("lse_finalize(Tensor m, Tensor s, Tensor? e, float s_total, float y_std, bool lse_out) "
        "-> (Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(dgprf, CUDA, m) {
  m.impl("sghmc_step_", &sghmc_step_);
  m.impl("potential_grad", &potential_grad);
  m.impl("forward", &forward);
  m.impl("forward_samples", &forward_samples);
  m.impl("lse_finalize", &lse_finalize);
}
