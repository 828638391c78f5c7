// capi_asan.cpp — host-side checks of libdgprf's C-ABI (include/dgprf.h) under AddressSanitizer +
// UndefinedBehaviorSanitizer (SURVEY §5 "ASan host tests").  Built by `make -C dgp-rf-mcmc_amd/csrc
// asan`: api.hip (plan derivation, argument validation, graph bookkeeping) compiled with
// -fsanitize=address,undefined on the host side only, linked with the other (uninstrumented)
// kernel objects into this executable.  No GPU is needed: every call here returns before any HIP
// runtime call — plan_init is host arithmetic, and each entry point validates its arguments first
// (the contract tests/test_capi.py checks through ctypes).  Exit status 0 = every check passed and
// the sanitizers reported nothing (a report aborts with a non-zero status).
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/dgprf.h"

static int failures = 0;
#define CHECK(cond)                                                           \
  do {                                                                        \
    if (!(cond)) {                                                            \
      std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #cond); \
      ++failures;                                                             \
    }                                                                         \
  } while (0)

static dgprf_plan_t make(int L, int d_in, int d_out, const int* kind, const int* n_rf,
                         const int* n_gp, int batch, int chains, int input_cat = 0,
                         int lik = DGPRF_LIK_GAUSSIAN) {
  dgprf_plan_t p;
  std::memset(&p, 0, sizeof(p));
  p.n_layers = L;
  p.d_in = d_in;
  p.d_out = d_out;
  p.input_cat = input_cat;
  p.likelihood = lik;
  p.batch = batch;
  p.n_chains = chains;
  p.hyp_flags = DGPRF_HYP_KERNEL | DGPRF_HYP_LIK;
  for (int l = 0; l < L && l < DGPRF_MAX_LAYERS; ++l) {
    p.kind[l] = kind[l];
    p.n_rf[l] = n_rf[l];
    p.n_gp[l] = n_gp[l];
    p.ard[l] = 1;
  }
  return p;
}

// Invariants of a derived plan: offsets inside the per-chain workspace, 4-float aligned, widths
// chained as models/dgp.py:76-79 builds them.
static void check_layout(const dgprf_plan_t& p) {
  CHECK(p.initialised == 1);
  CHECK(p.ws_chain > 0 && p.ws_total == p.ws_chain * p.n_chains);
  const int64_t offs[] = {p.gwp_off, p.logp_off, p.hpl_off, p.xb_off, p.yb_off};
  for (int64_t o : offs) CHECK(o >= 0 && o < p.ws_chain && o % 4 == 0);
  for (int l = 0; l < p.n_layers; ++l) {
    CHECK(p.d[l] == (l == 0 ? p.d_in : p.n_gp[l - 1] + (p.input_cat ? p.d_in : 0)));
    CHECK(p.P[l] == (p.kind[l] == DGPRF_RBF ? 2 : 1) * p.n_rf[l]);
    CHECK(p.w_off[l] % 4 == 0 && p.omega_off[l] % 4 == 0 && p.fp_off[l] % 4 == 0);
    CHECK(p.fp_off[l] < p.ws_chain && p.hpp_off[l] < p.ws_chain);
    CHECK(p.ns[l] >= 1 && p.ns[l] <= 16 && p.cpw[l] >= 1);
    CHECK((int64_t)p.ns[l] * p.cpw[l] * 64 >= p.n_rf[l]);
    if (l + 1 < p.n_layers) CHECK(p.w_off[l + 1] >= p.w_off[l] + (int64_t)p.P[l] * p.n_gp[l]);
  }
  CHECK(p.n_gw_rows >= 1 && p.n_gw_rows <= p.n_rt_pad && p.n_rt_pad % 16 == 0);
  CHECK(p.rt_per_group >= 1 && p.n_row_tiles == (p.batch + 15) / 16);
  if (p.a0_off >= 0) CHECK(p.d[0] > 32 && p.a0_off < p.ws_chain);
  if (p.omf_off >= 0) CHECK(p.fresh_z != 0 && p.omf_off < p.ws_chain);
  for (int64_t n : {(int64_t)0, (int64_t)1, (int64_t)1000, (int64_t)100000, (int64_t)10000000}) {
    int64_t need = -1;
    CHECK(dgprf_forward_scratch(&p, n, &need) == DGPRF_OK && need >= 0);
    for (int32_t S : {1, 2, 3, 20}) {
      int64_t need_s = -1;
      CHECK(dgprf_forward_samples_scratch(&p, n, S, &need_s) == DGPRF_OK && need_s >= need);
    }
  }
}

int main() {
  CHECK(dgprf_abi_version() == DGPRF_ABI_VERSION);
  for (int c : {DGPRF_OK, DGPRF_E_ARG, DGPRF_E_SHAPE, DGPRF_E_HIP, DGPRF_E_PLAN, 12345})
    CHECK(dgprf_error_string(c) != nullptr && std::strlen(dgprf_error_string(c)) > 0);

  // BASELINE.json configs 1-5 (and variants) over batch sizes and chain counts
  struct Cfg {
    int L, d_in, d_out, lik, cat;
    int kind[8], n_rf[8], n_gp[8];
  };
  const int R = DGPRF_RBF, A = DGPRF_ARC;
  const std::vector<Cfg> cfgs = {
      {1, 1, 1, DGPRF_LIK_GAUSSIAN, 0, {R}, {100}, {1}},
      {3, 8, 1, DGPRF_LIK_GAUSSIAN, 0, {R, R, R}, {1024, 1024, 1024}, {8, 8, 1}},
      {3, 9, 1, DGPRF_LIK_GAUSSIAN, 0, {A, A, A}, {2048, 2048, 2048}, {9, 9, 1}},
      {4, 784, 10, DGPRF_LIK_SOFTMAX, 0, {R, R, R, R}, {4096, 4096, 4096, 4096}, {30, 30, 30, 10}},
      {5, 16, 1, DGPRF_LIK_GAUSSIAN, 0, {R, A, R, A, R}, {8192, 8192, 8192, 8192, 8192},
       {16, 16, 16, 16, 1}},
      {2, 5, 3, DGPRF_LIK_SOFTMAX, 1, {A, R}, {33, 130}, {17, 3}},
      {8, 3, 2, DGPRF_LIK_GAUSSIAN, 1, {R, A, R, A, R, A, R, A}, {7, 9, 64, 65, 128, 1, 2, 300},
       {2, 3, 64, 1, 5, 6, 7, 2}},
  };
  int n_plans = 0;
  for (const Cfg& c : cfgs)
    for (int B : {1, 15, 16, 17, 200, 256, 257, 1024, 8192, 65536})
      for (int C : {1, 3, 64}) {
        if ((int64_t)B * C > 1 << 20) continue;
        dgprf_plan_t p = make(c.L, c.d_in, c.d_out, c.kind, c.n_rf, c.n_gp, B, C, c.cat, c.lik);
        const int rc = dgprf_plan_init(&p);
        CHECK(rc == DGPRF_OK || rc == DGPRF_E_SHAPE);  // 32-bit offset limits may refuse a shape
        if (rc == DGPRF_OK) {
          check_layout(p);
          ++n_plans;
          // options on a valid plan: fresh z, per-tile backward, forward paths, chunked A_1
          dgprf_plan_t q = p;
          q.fresh_z = (1 << c.L) - 1;
          q.bwd_tiles = 1;
          q.fwd_path = DGPRF_FWD_ROWS8;
          q.agemm_chunk_rows = 100;
          q.hyp_per_chain = 1;
          q.ard[0] = 0;
          const int rq = dgprf_plan_init(&q);
          CHECK(rq == DGPRF_OK || rq == DGPRF_E_SHAPE);
          if (rq == DGPRF_OK) check_layout(q);
        }
      }
  CHECK(n_plans > 100);

  // invalid plans are refused with a code, never by a crash
  const int k1[8] = {R}, r1[8] = {10}, g1[8] = {1};
  {
    dgprf_plan_t p = make(0, 1, 1, k1, r1, g1, 10, 1);
    CHECK(dgprf_plan_init(&p) == DGPRF_E_SHAPE);
    p = make(9, 1, 1, k1, r1, g1, 10, 1);
    CHECK(dgprf_plan_init(&p) == DGPRF_E_SHAPE);
    p = make(1, 1, 1, k1, r1, g1, 0, 1);
    CHECK(dgprf_plan_init(&p) == DGPRF_E_SHAPE);
    p = make(1, 1, 1, k1, r1, g1, 10, 0);
    CHECK(dgprf_plan_init(&p) == DGPRF_E_SHAPE);
    const int g65[8] = {65}, r0[8] = {0}, bad_kind[8] = {7};
    p = make(1, 1, 1, k1, r1, g65, 10, 1);
    CHECK(dgprf_plan_init(&p) == DGPRF_E_SHAPE);
    p = make(1, 1, 1, k1, r0, g1, 10, 1);
    CHECK(dgprf_plan_init(&p) == DGPRF_E_SHAPE);
    p = make(1, 1, 1, bad_kind, r1, g1, 10, 1);
    CHECK(dgprf_plan_init(&p) == DGPRF_E_ARG);
    p = make(1, 5000, 1, k1, r1, g1, 10, 1);
    CHECK(dgprf_plan_init(&p) == DGPRF_E_SHAPE);
    p = make(1, 1, 1, k1, r1, g1, 10, 1, 0, 9);
    CHECK(dgprf_plan_init(&p) == DGPRF_E_ARG);
    p = make(1, 1, 1, k1, r1, g1, 10, 1);
    p.fresh_z = 2;  // layer 1 of a 1-layer model
    CHECK(dgprf_plan_init(&p) == DGPRF_E_ARG);
    p = make(1, 1, 1, k1, r1, g1, 10, 1);
    p.bwd_tiles = 2;
    CHECK(dgprf_plan_init(&p) == DGPRF_E_ARG);
    p = make(1, 1, 1, k1, r1, g1, 10, 1);
    p.hyp_flags = 64;
    CHECK(dgprf_plan_init(&p) == DGPRF_E_ARG);
    p = make(1, 1, 1, k1, r1, g1, 10, 1);
    p.ard[0] = 2;
    CHECK(dgprf_plan_init(&p) == DGPRF_E_ARG);
    p = make(1, 1, 1, k1, r1, g1, 10, 1);
    p.fwd_path = 99;
    CHECK(dgprf_plan_init(&p) == DGPRF_E_ARG);
    p = make(1, 1, 1, k1, r1, g1, 10, 1);
    p.agemm_chunk_rows = -1;
    CHECK(dgprf_plan_init(&p) == DGPRF_E_ARG);
    CHECK(dgprf_plan_init(nullptr) == DGPRF_E_ARG);
  }

  // entry points validate before anything is enqueued (no device is touched)
  dgprf_plan_t ok = make(1, 1, 1, k1, r1, g1, 10, 1);
  CHECK(dgprf_plan_init(&ok) == DGPRF_OK);
  dgprf_plan_t uninit = ok;
  uninit.initialised = 0;
  float f = 0.f;
  int64_t i64 = 0;
  dgprf_chain_t ch;
  std::memset(&ch, 0, sizeof(ch));
  dgprf_batch_t bt;
  std::memset(&bt, 0, sizeof(bt));
  dgprf_step_t st;
  std::memset(&st, 0, sizeof(st));
  CHECK(dgprf_sghmc_step(&uninit, &ch, &bt, &st, nullptr) == DGPRF_E_PLAN);
  CHECK(dgprf_sghmc_step(&ok, nullptr, &bt, &st, nullptr) == DGPRF_E_ARG);
  CHECK(dgprf_sghmc_step(&ok, &ch, &bt, &st, nullptr) == DGPRF_E_ARG);  // null chain buffers
  ch.theta = ch.mom = ch.omega = ch.der = &f;
  ch.mass = &f;
  ch.ws = &f;
  ch.step = &i64;
  CHECK(dgprf_sghmc_step(&ok, &ch, &bt, &st, nullptr) == DGPRF_E_ARG);  // null batch rows
  bt.X = bt.Y = &f;
  bt.y_cols = 1;
  bt.n_data = 5;  // < batch
  CHECK(dgprf_sghmc_step(&ok, &ch, &bt, &st, nullptr) == DGPRF_E_SHAPE);
  bt.n_data = 100;
  bt.mode = 7;
  CHECK(dgprf_sghmc_step(&ok, &ch, &bt, &st, nullptr) == DGPRF_E_ARG);
  bt.mode = DGPRF_BATCH_EPOCH;
  bt.iters_per_epoch = 0;
  CHECK(dgprf_sghmc_step(&ok, &ch, &bt, &st, nullptr) == DGPRF_E_SHAPE);
  bt.mode = DGPRF_BATCH_INDEXED;  // without idx
  CHECK(dgprf_sghmc_step(&ok, &ch, &bt, &st, nullptr) == DGPRF_E_ARG);
  bt.mode = DGPRF_BATCH_DIRECT;
  CHECK(dgprf_sghmc_step(&ok, &ch, &bt, &st, nullptr) == DGPRF_E_ARG);  // data_size 0
  st.data_size = 100.f;
  st.schedule = 9;
  CHECK(dgprf_sghmc_step(&ok, &ch, &bt, &st, nullptr) == DGPRF_E_ARG);
  st.schedule = DGPRF_SCHED_CONST;
  st.full_bayes = 1;  // without z / hyp / hmom / hmass
  CHECK(dgprf_sghmc_step(&ok, &ch, &bt, &st, nullptr) == DGPRF_E_ARG);
  st.full_bayes = 0;
  CHECK(dgprf_potential_grad(&ok, &ch, &bt, 100.f, 0, nullptr, nullptr) == DGPRF_E_ARG);
  CHECK(dgprf_potential_grad(&ok, &ch, &bt, 0.f, 0, &f, nullptr) == DGPRF_E_ARG);
  dgprf_graph_handle h = reinterpret_cast<dgprf_graph_handle>(&f);
  CHECK(dgprf_graph_create_sghmc(nullptr, &ok, &ch, &bt, &st, 4) == DGPRF_E_ARG);
  CHECK(dgprf_graph_create_sghmc(&h, &ok, &ch, &bt, &st, 0) == DGPRF_E_ARG && h == nullptr);
  st.xi = &f;  // injected noise is not capturable
  CHECK(dgprf_graph_create_sghmc(&h, &ok, &ch, &bt, &st, 4) == DGPRF_E_ARG);
  st.xi = nullptr;
  CHECK(dgprf_graph_launch(nullptr, nullptr) == DGPRF_E_ARG);
  CHECK(dgprf_graph_destroy(nullptr) == DGPRF_OK);
  float ms[20];
  CHECK(dgprf_profile_step(&ok, &ch, &bt, &st, 0, ms, nullptr) == DGPRF_E_ARG);
  CHECK(dgprf_profile_step(&ok, &ch, &bt, &st, 5, nullptr, nullptr) == DGPRF_E_ARG);
  CHECK(dgprf_forward_scratch(&ok, -1, &i64) == DGPRF_E_ARG);
  CHECK(dgprf_forward_scratch(&uninit, 10, &i64) == DGPRF_E_PLAN);
  CHECK(dgprf_forward_samples_scratch(&ok, 10, 0, &i64) == DGPRF_E_ARG);
  CHECK(dgprf_forward_samples_scratch(&ok, -1, 2, &i64) == DGPRF_E_ARG);
  CHECK(dgprf_forward_samples_scratch(&ok, 10, 2, nullptr) == DGPRF_E_ARG);
  CHECK(dgprf_forward_samples_scratch(&uninit, 10, 2, &i64) == DGPRF_E_PLAN);
  CHECK(dgprf_forward(&ok, nullptr, &f, &f, &f, &f, 1, 10, nullptr, nullptr, nullptr, nullptr,
                      nullptr, nullptr, nullptr, 0, nullptr) == DGPRF_E_ARG);
  CHECK(dgprf_forward(&ok, &f, &f, &f, &f, nullptr, 1, 10, nullptr, &f, nullptr, nullptr,
                      nullptr, nullptr, nullptr, 0, nullptr) == DGPRF_E_ARG);  // log p without Y
  CHECK(dgprf_forward(&ok, &f, &f, &f, &f, &f, 1, 10, nullptr, nullptr, nullptr, &f, nullptr,
                      nullptr, nullptr, 0, nullptr) == DGPRF_E_ARG);  // lse_m without lse_s
  CHECK(dgprf_forward_samples(&ok, &f, 0, &f, &f, &f, nullptr, &f, 1, 10, &f, &f, nullptr,
                              nullptr, 0, nullptr) == DGPRF_E_ARG);
  CHECK(dgprf_forward_samples(&ok, &f, 2, &f, &f, &f, nullptr, &f, 1, 10, nullptr, &f, nullptr,
                              nullptr, 0, nullptr) == DGPRF_E_ARG);
  CHECK(dgprf_forward_samples(&ok, &f, 2, &f, &f, &f, nullptr, &f, 1, 10, &f, &f, nullptr,
                              nullptr, -1, nullptr) == DGPRF_E_ARG);
  {  // a resident A_1 with per-chain hyper-parameters over several chains (one Omega_1 each)
    const int kw[1] = {DGPRF_RBF}, rw[1] = {64}, gw[1] = {1};
    dgprf_plan_t pc = make(1, 40, 1, kw, rw, gw, 10, 2);
    pc.hyp_per_chain = 1;
    CHECK(dgprf_plan_init(&pc) == DGPRF_OK && pc.a0_off >= 0);
    CHECK(dgprf_forward_samples(&pc, &f, 2, &f, &f, &f, &f, &f, 1, 10, &f, &f, nullptr,
                                nullptr, 0, nullptr) == DGPRF_E_ARG);
  }
  CHECK(dgprf_lse_finalize(&f, &f, nullptr, 0, 10, 1.0, 0.f, 1.f, nullptr, nullptr, nullptr) ==
        DGPRF_E_ARG);
  CHECK(dgprf_rf_omega(9, 1, 1, &f, &f, &f, &f, &f, &f, nullptr) == DGPRF_E_ARG);
  CHECK(dgprf_rf_features(DGPRF_RBF, &f, -1, 1, &f, 1, &f, &f, nullptr) == DGPRF_E_ARG);
  CHECK(dgprf_gp_matmul(&f, 1, 1, &f, 0, &f, nullptr) == DGPRF_E_ARG);
  CHECK(dgprf_philox_normal(&f, 1, 1, 1, 300, nullptr) == DGPRF_E_ARG);
  CHECK(dgprf_philox_normal(nullptr, 1, 1, 1, 1, nullptr) == DGPRF_E_ARG);
  CHECK(dgprf_omega_build(&uninit, &f, &f, &f, &f, nullptr) == DGPRF_E_PLAN);
  CHECK(dgprf_omega_build(&ok, nullptr, &f, &f, &f, nullptr) == DGPRF_E_ARG);
  CHECK(dgprf_prior_w(&uninit, &f, &f, nullptr) == DGPRF_E_PLAN);

  if (failures) {
    std::fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  std::printf("capi_asan: %d plans derived, every check passed\n", n_plans);
  return 0;
}
