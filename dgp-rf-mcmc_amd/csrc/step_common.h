// step_common.h — types and device helpers shared by the step kernels' translation units
// (step_fwd_k*.hip, step_bwd_k*.hip, step_kernels.hip).
//
// Replaces DGP_RF.sgmcmc_update (models/dgp.py:184-216) with full_bayesian=False:
//   forward   per layer l:  Omega_l x -> c*[cos|sin] (RBF) or c*relu (ARC) -> Phi_l W_l
//             (layers/rf_layers.py:29-45,75-91; layers/GP_weight_layers.py:11-15; utils.py:10-44)
//   likelihood + potential U (likelihoods/gaussian.py:18-25, softmax.py:8-15, models/dgp.py:161-182)
//   backward  (analytic form of tape.gradient, models/dgp.py:194-198)
//   update    m <- b m - h N g + sqrt(2(1-b) T M) xi ; theta <- theta + h m / M (models/dgp.py:206-216)
//
// Decomposition (one chain = one blockIdx.z):
//   a workgroup owns a 16-row batch tile x a slice of RF features of one layer; each of its 4 waves
//   owns 16-feature chunks.  Contractions run on v_mfma_f32_16x16x4_f32 (exact fp32):
//     A^T[f][b]  = Omega^T X^T            (K = d_l)
//     F^T[o][b] += W^T Phi^T              (K = features, Phi straight from the A accumulator)
//     gW[f][o]   = Phi^T dF               (K = batch rows; A recomputed in row-major orientation)
//     dPhi[f][b] = W dF^T                 (K = g_l)
//     dX^T[k][b] = Omega dA^T             (K = features)
//   Cross-slice sums of F / dX partials are done by the CONSUMING kernel's prologue: always
//   DGPRF_NS_MAX slices (unused ones are zero) as one unrolled burst of independent loads summed in
//   a fixed order — deterministic, no atomics, one memory round trip.  The gW partials of the row
//   tiles are summed the same way by the update kernel, which also applies the prior term W/N and
//   the SGHMC update with Philox noise.
//
// Latency discipline (this path is latency-bound): every kernel gets a compact
// host-precomputed argument block (one round of independent scalar loads, no plan indexing);
// fragment loads are unconditional with clamped addresses (no exec-masked branches or per-load
// waits) and are issued before the dependent partial sums; minibatch rows of step t+1 are gathered
// by step t's update kernel, so the forward never waits on the step counter or the permutation.
#pragma once
#include <cstring>

#include "dgprf_internal.h"

namespace dgprf_sk {

constexpr int NW = DGPRF_WAVES;
constexpr int TR = DGPRF_TILE_ROWS;
constexpr int NSM = DGPRF_NS_MAX;
constexpr float LOG_2PI = 1.8378770664093453f;
constexpr int OST = 68;  // LDS row stride of the staged Omega block (16B-aligned rows)
// Row stride of the gW partial rows (floats): w_total plus this padding, so the rows a lane of the
// update kernel reads (configs 4 / 5: w_total x 4 B = 0x320000 / 0x310000 apart) do not share
// their low address bits
// Chains per launch from which a plan with <= 16 row tiles takes the row-group backward with one
// row group per chain (dgprf_plan_init)
#ifndef DGPRF_MC_RG_CHAINS
#define DGPRF_MC_RG_CHAINS 16
#endif
#ifndef DGPRF_GW_PAD
#define DGPRF_GW_PAD 0
#endif
__host__ __device__ inline int64_t gw_row_stride(int64_t w_total) { return w_total + DGPRF_GW_PAD; }

__host__ __device__ __forceinline__ int round4(int x) { return (x + 3) & ~3; }

// In-kernel timestamps of the per-tile step kernels, diagnostic -DDGPRF_STAMPS build only: into the
// buffer the launcher passes in a.stamps (16 slots per base; 15 / 13 = real time at slots 0 / 14).
#ifdef DGPRF_STAMPS
#define STEP_STAMP(base, i)                                                              \
  do {                                                                                   \
    if (threadIdx.x == 0 && a.stamps && (size_t)(base) < (size_t)17 * 4096) {             \
      __builtin_amdgcn_sched_barrier(0);                                                 \
      a.stamps[(size_t)(base) * 16 + (i)] = __builtin_amdgcn_s_memtime();                \
      if ((i) == 0) a.stamps[(size_t)(base) * 16 + 15] = __builtin_amdgcn_s_memrealtime(); \
      if ((i) == 14) a.stamps[(size_t)(base) * 16 + 13] = __builtin_amdgcn_s_memrealtime(); \
      __builtin_amdgcn_sched_barrier(0);                                                 \
    }                                                                                    \
  } while (0)
#else
#define STEP_STAMP(base, i) \
  do {                      \
    (void)(base);           \
  } while (0)
#endif

// Arguments of one forward / backward launch of layer `layer` (host-precomputed).
struct LayerK {
  const float* om;      // Omega_l [d][R] of chain 0 (chain stride om_cs; 0 = shared)
  const float* W;       // W_l [P][g] of chain 0 (chain stride w_cs)
  const float* fprev;   // F_{l-1} partials [NSM][B][gp] of chain 0 (chain stride ws_cs)
  float* fout;          // F_l partials [NSM][B][g]
  const float* dxnext;  // dX_{l+1} partials [NSM][B][g]        (backward, l < L-1)
  float* dxout;         // dX_l partials [NSM][B][dxw]           (backward, l > 0)
  float* gwp;           // gW partials of W_l, row-tile stride gw_ld (backward)
  float* logp;          // per-row log p [B]                       (backward, last layer)
  const float* xrows;   // minibatch X rows [B][d_in] (chain stride xrow_cs)
  const float* yrows;   // minibatch Y rows [B][y_cols] (chain stride yrow_cs)
  const float* cptr;    // c_l
  const float* varptr;  // sigma^2
  int64_t w_cs, ws_cs, xrow_cs, yrow_cs, om_cs, der_cs, gw_ld;
  int32_t d, R, g, gp, dxw, cpw, B, d_in, y_cols;
  int32_t last, likelihood, layer;
  int32_t xst, aux_off, auxst, red_off;
  int32_t stg_off, os_off;       // backward operand staging: W rows [2][64*g], Omega rows [.][OST]
  // element-owner prologue (fast == 1): workspace offsets of the partial buffers, magic divisors
  const float* ws;      // chain 0 workspace (chain stride ws_cs)
  int32_t fast, fprev_off, dsrc_off, xmag, dmag;
  int32_t n_rt, ns, rt_per_xcd;  // XCD-aware block -> (row tile, slice) map
  // full_bayesian=True (k_step_bwd<..., FB = true>)
  const float* a0;      // precomputed A_1 [align32(B)][R] (layer 0 with d > 32; chain stride
                        // ws_cs), nullptr otherwise
  const float* z;       // z_l [d][R] (shared by the chains)
  float* hp;            // hyper partials [n_rt_pad][NSM][round4(2d+1)] of chain 0 (stride ws_cs)
  float* hpl;           // lik_log_var partials [n_rt_pad] (last layer)
  int32_t hred_off, lik_fb;
  // whole-slice staging (backward, cpw >= 4): the workgroup's W rows [h][64 cpw][g] and Omega rows
  // [dxw][64 cpw + 4] are copied global -> LDS once (global_load_lds) instead of one 64-feature
  // block per chunk with a load round trip and two barriers each
  int32_t wstage, wsa_off, osa_off, osa_st, kind_rbf;
  // per-tile backward, 1 < g with g % 16 != 0: per-wave gW staging [nwb][2][16][g] (0: none)
  int32_t gst_off;
  int32_t main_blocks;  // this layer's (row tile, slice) workgroups
  int32_t a0_sl;  // layer 0 with a0: second K-part slab of A_1 at a0 + a0_sl (0: one slab)
  // row-group backward (k_step_bwd_rg, minibatches of > 16 row tiles): rt_per_rg row tiles per
  // workgroup, ncw chunk-waves x nrw row-waves, register-prefetched prologue when rg_fast
  int32_t rt_per_rg, ncw, nrw, rg_fast, gred_off, rg_nit;
  int32_t rw_orows, rw_pad;  // row-wave backward: staged Omega rows (zero past d)
  int32_t rw_one;         // row-wave backward: the dF source is one complete slice (= last)
  int32_t cmp;           // row-group backward after the fused forward (step_fused_fwd): every
                         // F_l is complete in slice 0 of its partial buffer (one load, not 16)
  int32_t rcf, rcf_off;  // output layer folded into its backward (step_fold_out): the layer's
                         // whole W_L [P] and Omega_L [d][R + 16] staged in LDS at rcf_off
  unsigned long long* stamps;  // -DDGPRF_STAMPS diagnostic build: stamp buffer, else null
};

// A_1 elements at p: slab 0 + slab 1 of the GEMM's two K parts (sl = 0: one slab).  Every layer-0
// consumer adds them in this order, so the forward and the backward see the same A_1.
__device__ __forceinline__ f4 a0_sum4(const float* p, int sl) {
  f4 v = *reinterpret_cast<const f4*>(p);
  if (sl) v += *reinterpret_cast<const f4*>(p + sl);
  return v;
}
__device__ __forceinline__ float a0_sum1(const float* p, int sl) { return sl ? p[0] + p[sl] : p[0]; }

// Block -> (row tile, slice): blocks are dealt round-robin over the 8 XCDs, so block b's XCD group
// is b % 8; every workgroup of row tile rt gets group rt % 8, so the slice partials it exchanges
// with the neighbouring layers' kernels stay within one L2.  Speed only: correctness never depends
// on placement.  Blocks past the last row tile exit at once.
// rt_per_xcd == 0: a plain row-major map (rt = b / ns) — several chains per launch with fewer than
// 8 row tiles / groups each, where the XCD map would leave XCDs idle (every chain's blocks start at
// a multiple of 8).
__device__ __forceinline__ bool tile_of_block(const LayerK& a, int& rt, int& sl) {
  if (a.rt_per_xcd == 0) {
    rt = (int)blockIdx.x / a.ns;
    sl = (int)blockIdx.x - rt * a.ns;
    return rt < a.n_rt;
  }
  const int b = blockIdx.x, grp = b & 7, idx = b >> 3;
  const int j = idx / a.ns;
  sl = idx - j * a.ns;
  rt = grp + 8 * j;
  return rt < a.n_rt;
}

// full_bayesian=True hyper-parameter work, run by extra one-wave workgroups of k_step_update
// (models/dgp.py:175-181, 199-216).  Layer l owns nb[l] workgroups starting at b0[l] (one each in
// gradient-only mode); the last hyper workgroup handles the Gaussian lik_log_var.
struct HypK {
  float* hyp;          // chain 0 (chain stride hyp_cs)
  float* hmom;         // [C][hyp_total]
  const float* hmass;  // [C][DGPRF_HMASS]
  const float* z;
  float* omega;        // chain 0 (chain stride om_cs)
  float* der;          // chain 0 (chain stride der_cs)
  const float* ws;     // chain 0 workspace (chain stride ws_cs of UpdK)
  int64_t hyp_cs, om_cs, der_cs, hyp_total, cnt_off;
  int32_t n_blocks, flags, likelihood, pad;
  int32_t d[DGPRF_MAX_LAYERS], R[DGPRF_MAX_LAYERS], kind[DGPRF_MAX_LAYERS], ard[DGPRF_MAX_LAYERS];
  int32_t ns[DGPRF_MAX_LAYERS], nb[DGPRF_MAX_LAYERS], b0[DGPRF_MAX_LAYERS];
  int64_t lis_off[DGPRF_MAX_LAYERS], mean_off[DGPRF_MAX_LAYERS], om_off[DGPRF_MAX_LAYERS];
  int64_t hpp_off[DGPRF_MAX_LAYERS], hpl_off;
};

// Arguments of the update kernel (hot fields first: one burst of scalar loads).
struct UpdK {
  float* theta;         // chain 0 (chain stride w_total)
  float* mom;
  const float* gwp;     // gW partials base of chain 0 (chain stride ws_cs, row-tile stride gw_ld)
  const float* mass;
  const int64_t* step;
  int32_t w_total, n_rt, n_rt_pad, n_layers;
  int32_t lo[DGPRF_MAX_LAYERS], hi[DGPRF_MAX_LAYERS];
  int32_t gw_ld, pad_g;  // gW partial row stride (gw_row_stride)
  uint64_t seed;
  int64_t ws_cs;
  int32_t step_offset, upd_blocks;
  int32_t e_end, pad_e;  // parameters [0, e_end) are updated (e_end < w_total: the first layers only)
  UpdateDev ud;
  const float* grad_in;
  float* grad_out;
  int64_t grad_cs;      // chain stride of grad_out (w_total, or w_total + hyp_total in full Bayes)
  // gather of step t+1's minibatch rows (graph mode)
  int32_t gather_next, B, d_in, yb_cols;
  BatchDev bd;
  float* xb;
  float* yb;
  float* a0;  // resident A_1 rows of step t+1 (bd.A1): the workspace slab, chain 0
  int32_t gather_blocks, a1_parts;
  // full_bayesian=True: the first hyp_blocks workgroups do the hyper-parameter work
  int32_t hyp_blocks, pad_h;
  HypK hk;
  // eager steps: arrival counter of the workgroups, the last one advancing *step (else null)
  unsigned* adv_cnt;
  int64_t* step_adv;
};

// v if ok else 0, written so that the compiler cannot sink the (always in-range, finite) load
// into an exec-masked branch followed by an immediate wait: the load result is used on every path.
__device__ __forceinline__ float keep(float v, bool ok) { return v * (ok ? 1.f : 0.f); }

// Sum over each 16-lane row of the wave (ds_swizzle xor butterflies, fixed order; every lane of
// the row ends with the same value).
template <int XM>
__device__ __forceinline__ float swz_xor(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, v),
                                                               (XM << 10) | 0x1F));
}
__device__ __forceinline__ float sum16(float v) {
  v += swz_xor<8>(v);
  v += swz_xor<4>(v);
  v += swz_xor<2>(v);
  v += swz_xor<1>(v);
  return v;
}

// sum over the DGPRF_NS_MAX slices of a partial buffer: independent loads, fixed order.
__device__ __forceinline__ float sum_slices(const float* __restrict__ p, int64_t stride) {
  float v[NSM];
#pragma unroll
  for (int s = 0; s < NSM; ++s) v[s] = p[s * stride];
  float acc = v[0];
#pragma unroll
  for (int s = 1; s < NSM; ++s) acc += v[s];
  return acc;
}

// LDS layout of one forward / backward workgroup of nwb waves (floats): X tile [TR][xst], the
// backward's dF and Y tiles [TR][auxst], then `red` — the per-wave reduction rows (F [nwb][TR][GP + 4]
// in the forward, dX [nwb][TR][DP + 4] in the backward; also the prologue's scratch slots) — then the
// backward's 64-feature W / Omega staging block when dPhi / dX need them.  Sized to the layer, so
// small layers leave room for more resident workgroups (large minibatches).
__host__ __device__ inline void step_lds(LayerK& a, int& total, int nwb, bool bwd, bool dphi) {
  const int d = a.d, g = a.g;
  a.xst = round4(d) + 1;
  a.aux_off = round4(TR * a.xst);
  a.auxst = g + 1;
  a.red_off = a.aux_off + (bwd ? 2 * round4(TR * a.auxst) : 0);  // dF tile + Y tile
  const int np = 64 * nwb < 512 ? 64 * nwb : 512;       // prologue owners (scratch: 2 np slots)
  // reduction rows padded by 4 floats (conflict-free 16-byte row writes)
  const int gp16 = (g + 15) / 16 * 16 + 4, dp16 = (a.dxw + 15) / 16 * 16 + 4;
  const int rows = nwb * TR * (bwd ? dp16 : gp16);
  a.stg_off = a.red_off + round4(rows > 2 * np ? rows : 2 * np);
  if (bwd && dphi) {  // backward: the workgroup's 64-feature block of W_l ([2][64*g]), Omega_l ([64][OST])
    a.os_off = a.stg_off + (2 * 64 * g > 2048 ? round4(2 * 64 * g) : 2048);
    total = a.os_off + 64 * OST;
  } else {
    a.os_off = a.stg_off;
    total = a.stg_off;
  }
}

// floor(i / n) = (i * magic(n)) >> 20 for 0 <= i < 4096, 1 <= n <= 256
__host__ __device__ inline int div_magic(int n) { return (int)((1048576 + n - 1) / n); }

// X_l[16][d] of batch rows row0..: F_{l-1} partial sums (+ [F | X] dataset columns for input_cat,
// utils.py:42) or the gathered minibatch rows for layer 0.
__device__ __forceinline__ void load_x_tile(const LayerK& a, int chain, int row0, float* xs) {
  const int dpad = round4(a.d);
  const float* fprev = a.fprev + (int64_t)chain * a.ws_cs;
  const float* xr = a.xrows + (int64_t)chain * a.xrow_cs;
  for (int e = threadIdx.x; e < TR * dpad; e += blockDim.x) {
    const int r = e / dpad, k = e - r * dpad, b = row0 + r;
    const int bc = min(b, a.B - 1), kc = min(k, a.d - 1);
    float v;
    if (kc < a.gp)
      v = sum_slices(fprev + (int64_t)bc * a.gp + kc, (int64_t)a.B * a.gp);
    else
      v = xr[(int64_t)bc * a.d_in + (kc - a.gp)];
    xs[r * a.xst + k] = (b < a.B && k < a.d) ? v : 0.f;
  }
}

// ---- element-owner prologue (a.fast == 1).  Thread t owns tile elements u = t + 256p (p < 2):
// the X tile (TR x dpad: F_{l-1} slice partials | dataset columns) first, then, in the backward,
// the dF tile (TR x g: dX_{l+1} or F_L slice partials, with the matching Y value).  Every owned
// element issues its 16 slice loads on the chain's workspace plus one dataset / Y load; absent
// slices, rows >= B and padding columns get an out-of-range offset (0, no memory access).  All
// loads of the prologue are issued before the first sum, which runs in registers in the same fixed
// slice order as sum_slices.
struct Elem {
  float v[NSM];
  float xd, y;
  int dst;  // LDS index (xs / dfs), or -1
  bool isx;
};

__device__ __forceinline__ void elem_issue(const LayerK& a, int chain, int row0, int u,
                                           int nd_tile, int dfst, Elem& e) {
  const rsrc_t rws = make_rsrc(a.ws + (int64_t)chain * a.ws_cs, a.ws_cs);
  const rsrc_t rx = make_rsrc(a.xrows + (int64_t)chain * a.xrow_cs, (int64_t)a.B * (a.d - a.gp));
  const rsrc_t ry = make_rsrc(a.yrows + (int64_t)chain * a.yrow_cs, (int64_t)a.B * a.y_cols);
  const int dpad = round4(a.d), nx = TR * dpad, ndat = a.d - a.gp;
  const bool isx = u < nx, isd = !isx && u < nx + nd_tile;
  const int ud = u - nx;
  const int r = isx ? (u * a.xmag) >> 20 : (ud * a.dmag) >> 20;
  const int c = isx ? u - r * dpad : ud - r * a.g;
  const int b = row0 + r;
  const bool inb = b < a.B && (isx || isd);
  // (a folded output layer forms its F_L tile itself: only its Y values are loaded here)
  const bool fromp = inb && (isx ? c < a.gp : !a.rcf);
  const int w = isx ? a.gp : a.g;
  const int base = (isx ? a.fprev_off : a.dsrc_off) + b * w + c;
  const int str = a.B * w;
#pragma unroll
  for (int sl = 0; sl < NSM; ++sl)
    e.v[sl] = bload1(rws, fromp ? (uint32_t)((base + sl * str) * 4) : DGPRF_OOB);
  const bool xdat = inb && isx && c >= a.gp && c < a.d;
  e.xd = bload1(rx, xdat ? (uint32_t)((b * ndat + (c - a.gp)) * 4) : DGPRF_OOB);
  const int yc = a.likelihood == DGPRF_LIK_GAUSSIAN ? a.g : 1;
  const bool ydat = inb && isd && a.last;
  e.y = bload1(ry, ydat ? (uint32_t)((b * a.y_cols + min(c, yc - 1)) * 4) : DGPRF_OOB);
  e.isx = isx;
  e.dst = isx ? r * a.xst + c : (isd ? r * dfst + c : -1);
}
// sum + store: xs[dst] or dfs[dst] (and ysh[dst]); non-owning lanes write a scratch slot
__device__ __forceinline__ void elem_store(const Elem& e, float* xs, float* dfs, float* ysh,
                                          float* scratch, int np) {
  float acc = e.v[0];
#pragma unroll
  for (int sl = 1; sl < NSM; ++sl) acc += e.v[sl];
  const float val = e.isx ? acc + e.xd : acc;  // exactly one of the two is non-zero-sourced
  float* dv = e.dst < 0 ? scratch : (e.isx ? xs + e.dst : dfs + e.dst);
  float* dy = (e.dst < 0 || e.isx) ? scratch + np : ysh + e.dst;
  *dv = val;
  *dy = e.y;
}

// Element-owner prologue of one kernel: X tile (and dF tile when nd_tile > 0) into LDS.
__device__ __forceinline__ void elem_prologue(const LayerK& a, int chain, int row0, int nd_tile,
                                             float* xs, float* dfs, int dfst, float* ysh,
                                             float* scratch) {
  const int total = TR * round4(a.d) + nd_tile;
  const int t = threadIdx.x;
  const int np = min((int)blockDim.x, 512);  // owning threads: elements t and t + np
  if (t >= np) return;  // 16-wave workgroups: waves 0-7 own the elements (wave-uniform)
  const int wave0 = __builtin_amdgcn_readfirstlane(t & ~63);
  Elem e0, e1;
  if (wave0 < total) elem_issue(a, chain, row0, t, nd_tile, dfst, e0);
  if (np + wave0 < total) elem_issue(a, chain, row0, t + np, nd_tile, dfst, e1);
  if (wave0 < total) elem_store(e0, xs, dfs, ysh, scratch + t, np);
  if (np + wave0 < total) elem_store(e1, xs, dfs, ysh, scratch + t, np);
}

// The same prologue with `mid()` run between issuing the loads and their sums (every thread calls
// it: workgroups of <= 8 waves only) — the folded output layer issues its LDS copies of W_L /
// Omega_L there, so they queue behind the partial-sum loads instead of delaying them.
template <class Mid>
__device__ __forceinline__ void elem_prologue_mid(const LayerK& a, int chain, int row0, int nd_tile,
                                                  float* xs, float* dfs, int dfst, float* ysh,
                                                  float* scratch, Mid mid) {
  const int total = TR * round4(a.d) + nd_tile;
  const int t = threadIdx.x;
  const int np = (int)blockDim.x;  // <= 512
  const int wave0 = __builtin_amdgcn_readfirstlane(t & ~63);
  Elem e0, e1;
  if (wave0 < total) elem_issue(a, chain, row0, t, nd_tile, dfst, e0);
  if (np + wave0 < total) elem_issue(a, chain, row0, t + np, nd_tile, dfst, e1);
  mid();
  if (wave0 < total) elem_store(e0, xs, dfs, ysh, scratch + t, np);
  if (np + wave0 < total) elem_store(e1, xs, dfs, ysh, scratch + t, np);
}

// Omega fragments: omk[ks] = Omega[4ks+lq][f0+lr] (zero outside the layer), KS k-steps.
template <int KS>
__device__ __forceinline__ void load_om_frag(const float* __restrict__ om, int R, int d, int f0,
                                             int lr, int lq, float (&omk)[8]) {
  const int fa = f0 + lr;
  const int fc = min(fa, R - 1);
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int k = 4 * ks + lq;
    omk[ks] = keep(om[(int64_t)min(k, d - 1) * R + fc], fa < R && k < d);
  }
}

// A-tile.  TRANS=false: at[r] = A[row lr][f0+4lq+r] (features in regs)
//          TRANS=true : at[r] = A[row 4lq+r][f0+lr] (rows in regs)
template <int KS, bool TRANS>
__device__ __forceinline__ f4 a_tile(const float* __restrict__ om, int R, int d, int f0,
                                     const float (&omk)[8], const float (&xf)[8],
                                     const float* xs, int xst, int lr, int lq) {
  f4 at = f4zero();
  if (KS > 0) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      at = TRANS ? mfma16(xf[ks], omk[ks], at) : mfma16(omk[ks], xf[ks], at);
  } else {
    const int fa = f0 + lr, fc = min(fa, R - 1);
    const int nks = round4(d) >> 2;
    for (int ks = 0; ks < nks; ++ks) {
      const int k = 4 * ks + lq;
      const float ov = om[(int64_t)min(k, d - 1) * R + fc];
      const float o = (fa < R && k < d) ? ov : 0.f;
      const float x = xs[lr * xst + 4 * ks + lq];
      at = TRANS ? mfma16(x, o, at) : mfma16(o, x, at);
    }
  }
  return at;
}

template <bool RBF>
__device__ __forceinline__ void features(const f4 at, float cl, float (&p0)[4], float (&p1)[4]) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (RBF) {
      float s, c;
      rf_sincos(at[r], &s, &c);
      p0[r] = cl * c;
      p1[r] = cl * s;
    } else {
      p0[r] = cl * fmaxf(at[r], 0.f);
      p1[r] = 0.f;
    }
  }
}

// Omega[k][f] with both indices clamped into the [rows][R] block (always a valid address).
__device__ __forceinline__ float om_safe(const float* __restrict__ om, int R, int rows, int k,
                                         int f) {
  return om[(int64_t)min(k, rows - 1) * R + min(f, R - 1)];
}

// W fragments for F^T += W^T Phi^T: wf[ot][r][0|1] = W[f0+4lq+r (| R+...)][ot*16+lr] (G1: column
// 0 in every lane), clamped raw loads; the caller masks at the point of use (w_ok), so a prefetch
// never waits on its own loads.
template <int NOT, bool RBF, bool G1>
__device__ __forceinline__ void load_w_frag(const float* __restrict__ W, int R, int g, int f0,
                                            int lr, int lq, float (&wf)[NOT][4][2]) {
#pragma unroll
  for (int ot = 0; ot < NOT; ++ot) {
    const int oc = G1 ? 0 : min(ot * 16 + lr, g - 1);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int fc = min(f0 + 4 * lq + r, R - 1);
      wf[ot][r][0] = W[(int64_t)fc * g + oc];
      wf[ot][r][1] = RBF ? W[(int64_t)(R + fc) * g + oc] : 0.f;
    }
  }
}
template <bool G1>
__device__ __forceinline__ bool w_ok(int ot, int r, int R, int g, int f0, int lr, int lq) {
  return (G1 || ot * 16 + lr < g) && f0 + 4 * lq + r < R;
}

// ------------------------------------------------------------------------- update / gather
__device__ __forceinline__ f4 ld4(const float* p) { return *reinterpret_cast<const f4*>(p); }
__device__ __forceinline__ void st4(float* p, f4 v) { *reinterpret_cast<f4*>(p) = v; }

// cyclical_step_rate (utils.py:49-73) with min_value = 0 as used by the drivers
// (experiments/utils_training.py:53-54): lr = lr0 * rate^2.
__device__ __forceinline__ float cyclical_rate(int64_t step_index, int64_t cycle) {
  const float frac = (float)((step_index - 1) % cycle) / (float)cycle;
  return 0.0f + (1.0f - 0.0f) * 0.5f * (cosf(3.14159265358979f * frac) + 1.0f);
}

// Copy minibatch row b of chain `chain` at step t into the gathered-rows workspace.
__device__ __forceinline__ void gather_row(const BatchDev& bd, int B, int d_in, int yb_cols,
                                           float* xb, float* yb, int chain, int64_t t, int b) {
  const int64_t row = batch_row(bd, B, chain, t, b);
  const float* xs = bd.X + row * d_in;
  const float* ys = bd.Y + row * bd.y_cols;
  float* xd = xb + (int64_t)b * d_in;
  float* yd = yb + (int64_t)b * yb_cols;
  for (int k = 0; k < d_in; ++k) xd[k] = xs[k];
  for (int k = 0; k < yb_cols; ++k) yd[k] = ys[k];
}

// Wide rows (d_in > GATHER_WIDE, e.g. 784 MNIST pixels): one 64-lane wave per row, lanes striding
// over the columns (coalesced, all loads issued before the stores) instead of one thread per row.
constexpr int GATHER_WIDE = 16;
__device__ __forceinline__ void gather_row_wave(const BatchDev& bd, int B, int d_in, int yb_cols,
                                                float* xb, float* yb, int chain, int64_t t, int b,
                                                int lane) {
  const int64_t row = batch_row(bd, B, chain, t, b);
  const float* xs = bd.X + row * d_in;
  float* xd = xb + (int64_t)b * d_in;
  constexpr int U = 8;
  for (int k0 = 0; k0 < d_in; k0 += 64 * U) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + 64 * u + lane;
      v[u] = k < d_in ? xs[k] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + 64 * u + lane;
      if (k < d_in) xd[k] = v[u];
    }
  }
  for (int k = lane; k < yb_cols; k += 64) yb[(int64_t)b * yb_cols + k] = bd.Y[row * bd.y_cols + k];
}

// Resident first-layer projection (BatchDev.A1 = X Omega_1 of every dataset row): the 1,024-float
// part `part` of minibatch row b's A_1 row into the workspace slab [align32(B)][R_1] the layer-0
// kernels read — one wave, four 16-byte loads per lane issued before the stores.  Replaces the
// step's A_1 = X_B Omega_1 GEMM (the rows of a product are the products of the rows).
constexpr int A1_PART = 1024;
__device__ __forceinline__ void gather_a1_part(const BatchDev& bd, int B, float* a0, int chain,
                                               int64_t t, int b, int part, int lane) {
  const int64_t row = batch_row(bd, B, chain, t, b);
  const int R0 = bd.a1_ld;
  const float* src = bd.A1 + row * R0;
  float* dst = a0 + (int64_t)b * R0;
  f4 v[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int k = part * A1_PART + 4 * (u * 64 + lane);
    v[u] = k < R0 ? *reinterpret_cast<const f4*>(src + k) : f4zero();
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int k = part * A1_PART + 4 * (u * 64 + lane);
    if (k < R0) *reinterpret_cast<f4*>(dst + k) = v[u];
  }
}

// Schedule of step t (utils.py:49-73 via experiments/utils_training.py:41-61 when CYC).
template <bool CYC>
__device__ __forceinline__ void step_schedule(const UpdateDev& ud, int64_t t, float* lr, float* T,
                                              int* resample) {
  *lr = ud.lr;
  *T = ud.temperature;
  *resample = ud.resample;
  if (CYC) {
    if (t < ud.start_step) {  // burn-in: fixed lr, zero temperature
      *T = 0.f;
      *resample = 0;
    } else {
      const int64_t si = t - ud.start_step + 1;
      const float rate = cyclical_rate(si, ud.cycle_length);
      *lr = ud.lr * (rate * rate);
      *T = 1.f;
      *resample = ud.resample_head && (si % ud.cycle_length == 1);
    }
  }
}


// One lane's four packed parameters e0..e0+3 (one counter quad of Philox normals, 16-byte loads;
// layer offsets are multiples of 4, so a quad never straddles two layers): the row-tile gW partials
// summed in a fixed order, the prior term W/N, and m <- b m - h N g + sqrt(2(1-b) T M) xi,
// theta <- theta + h m / M (models/dgp.py:206-216).  Parameters past e_end (or a layer's end) are
// not stored.  GIN: gradient supplied (grad_in); GONLY: write the gradient (grad_out) instead.
// (A ride-along form — layer l + 1's W updated by extra workgroups of layer l's backward launch —
// measured slower: config 4 123.7 vs 116.3 us/step, config 5 98.0 vs 96.5)
template <bool GIN, bool GONLY, bool XI, bool CYC, class K>
__device__ __forceinline__ void w_update_quad(const K& a, const int e0, const int chain) {
  const uint32_t off = (uint32_t)e0 * 4u;
  const int64_t cw = (int64_t)chain * a.w_total;
  int layer = 0;
#pragma unroll
  for (int l = 1; l < DGPRF_MAX_LAYERS; ++l)
    if (l < a.n_layers && e0 >= a.lo[l]) layer = l;
  // the mass and the step counter (written by the previous graph's k_advance) are loaded together
  // with the parameters and partials: placed after the partial sums, the compiler issued them
  // only once those had been waited for — a second dependent memory round trip per step
  // layer padding between align4 offsets stays untouched: live elements of the quad (a.hi is
  // indexed per lane, so this too is a memory load: issued here, not after the sums)
  const int nlive = min(max(min(a.hi[layer], a.e_end) - e0, 0), 4);
  const float M = GONLY ? 1.f : a.mass[chain * a.n_layers + layer];
  const int64_t t = GONLY ? 0 : *a.step + (int64_t)a.step_offset;
  const rsrc_t rth = make_rsrc(a.theta + cw, a.w_total);
  const f4 th = bload4(rth, off);
  f4 m = f4zero(), gr;
  if (!GONLY) m = bload4(make_rsrc(a.mom + cw, a.w_total), off);
  if constexpr (GIN) {
    gr = bload4(make_rsrc(a.grad_in + cw, a.w_total), off);
  } else {
    // sum the row-tile gW partials in a fixed order: groups of 16 independent loads (rows past
    // n_rt read 0 through the descriptor bound and leave the sum unchanged).  One row (a row group
    // per chain) or <= 4 rows: only those loads — the 15 / 12 bound-clipped ones still pass
    // through the texture path (64 chains of config 4 / 5: 3,227 -> 3,188 / 3,542 -> 3,491 us)
    const rsrc_t rs = make_rsrc(a.gwp + (int64_t)chain * a.ws_cs, (int64_t)a.n_rt * a.gw_ld);
    f4 sacc = f4zero();
    if (a.n_rt == 1) {
      sacc = bload4(rs, off);
    } else if (a.n_rt <= 4) {
      f4 v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = bload4(rs, (uint32_t)((j * a.gw_ld + e0) * 4));
#pragma unroll
      for (int j = 0; j < 4; ++j) sacc += v[j];
    } else {
      for (int rt0 = 0; rt0 < a.n_rt_pad; rt0 += 16) {
        f4 v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = bload4(rs, (uint32_t)(((rt0 + j) * a.gw_ld + e0) * 4));
#pragma unroll
        for (int j = 0; j < 16; ++j) sacc += v[j];
      }
    }
    gr = sacc;
  }
  // theta / momenta / gradient stores (write-through stores here gained nothing: 116.1 vs 116.3,
  // 97.5 vs 97.2 us/step on configs 4 / 5)
  auto store = [&](float* base, f4 v) {  // base: the chain's array (w_total floats)
    float* p = base + e0;
    if (nlive == 4) {
      *reinterpret_cast<f4*>(p) = v;
    } else {
      for (int k = 0; k < nlive; ++k) p[k] = v[k];
    }
  };
  const UpdateDev& ud = a.ud;
  const float N = ud.data_size;
  // dU/dW = W/N (prior N(0,1), models/dgp.py:129-136,171) + Phi^T dF (likelihood)
  if (!GIN) gr = th / N + gr;
  if constexpr (GONLY) {
    store(a.grad_out + (int64_t)chain * a.grad_cs, gr);
    return;
  } else {
    float lr, T;
    int resample;
    step_schedule<CYC>(ud, t, &lr, &T, &resample);
    const float h = sqrtf(lr / N);
    const float beta = ud.beta;
    const uint32_t quad = (uint32_t)(e0 >> 2);
    if (resample) {  // models/dgp.py:209-210 (ignores M, Appendix A.1)
      if (XI && ud.xi_resample)  // lanes past w_total (the last block's tail) read 0, no access
        m = bload4(make_rsrc(ud.xi_resample + cw, a.w_total), off);
      else
        m = philox_normal4(a.seed, (uint64_t)t, DGPRF_RNG_RESAMPLE, (uint32_t)chain, quad);
    }
    f4 mn = beta * m - (h * N) * gr;
    const f4 eps = (XI && ud.xi) ? bload4(make_rsrc(ud.xi + cw, a.w_total), off)
                                 : philox_normal4(a.seed, (uint64_t)t, DGPRF_RNG_NOISE, (uint32_t)chain, quad);
    mn = mn + sqrtf(2.0f * (1.0f - beta) * T * M) * eps;
    store(a.mom + cw, mn);
    store(a.theta + cw, th + (h * (1.0f / M)) * mn);
  }
}

// Minimum waves per SIMD the register allocation must allow.  Single-chain steps run one workgroup
// per CU either way; with C chains per launch (13 x 16 x C workgroups) residency sets throughput:
// the g <= 16, d <= 8 W-only backward at <= 168 VGPRs (3 waves/SIMD) measured 127k -> 156k
// chain-steps/s at C = 64 and single-chain 36.3k -> 36.7k steps/s (config 3's ARC layers +3 %);
// the wider / full-Bayes instances keep their registers (they would spill 20-200 VGPRs; config 5's
// RBF d = 16 layers lost 8 % with 22 spilled).
constexpr int STEP_WPE = 3;

// (row tile | row group, slice) workgroups of one launch: the XCD-aware map, or the plain map for
// several chains with fewer than 8 row tiles / groups each (tile_of_block)
inline void set_block_map(LayerK& a, int n_rt, int n_chains) {
  a.n_rt = n_rt;
  if (n_chains > 1 && n_rt < 8) {
    a.rt_per_xcd = 0;
    a.main_blocks = n_rt * a.ns;
  } else {
    a.rt_per_xcd = (n_rt + 7) / 8;
    a.main_blocks = 8 * a.rt_per_xcd * a.ns;
  }
}

inline LayerK make_layer_k(const dgprf_plan_t& pl, const StepDev& sd, int l, int& lds_floats,
                    bool bwd = false, int nwb = NW) {
  LayerK a;
  const bool direct = sd.bd.mode == DGPRF_BATCH_DIRECT;
  // random_fixed=False layers read this step's Omega from the workspace (k_fresh_omega)
  const bool fresh = ((pl.fresh_z >> l) & 1) && pl.omf_off >= 0;
  a.om = fresh ? sd.ws + pl.omf_off + pl.omega_off[l] : sd.omega + pl.omega_off[l];
  a.W = sd.theta + pl.w_off[l];
  a.fprev = l > 0 ? sd.ws + pl.fp_off[l - 1] : sd.ws;
  a.fout = sd.ws + pl.fp_off[l];
  a.dxnext = l + 1 < pl.n_layers ? sd.ws + pl.dxp_off[l + 1] : sd.ws;
  a.dxout = l > 0 ? sd.ws + pl.dxp_off[l] : sd.ws;
  a.gwp = sd.ws + pl.gwp_off + pl.w_off[l];
  a.logp = sd.ws + pl.logp_off;
  a.xrows = direct ? sd.bd.X : sd.ws + pl.xb_off;
  a.yrows = direct ? sd.bd.Y : sd.ws + pl.yb_off;
  a.xrow_cs = direct ? 0 : pl.ws_chain;
  a.yrow_cs = direct ? 0 : pl.ws_chain;
  a.y_cols = direct ? sd.bd.y_cols : pl.yb_cols;
  a.cptr = sd.der + l;
  a.varptr = sd.der + DGPRF_MAX_LAYERS;
  a.om_cs = fresh ? pl.ws_chain : sd.om_cs;
  a.der_cs = sd.der_cs;
  a.w_cs = pl.w_total;
  a.gw_ld = gw_row_stride(pl.w_total);
  a.ws_cs = pl.ws_chain;
  a.d = pl.d[l];
  a.R = pl.n_rf[l];
  a.g = pl.n_gp[l];
  a.gp = l > 0 ? pl.n_gp[l - 1] : 0;
  a.dxw = l > 0 ? pl.n_gp[l - 1] : 0;
  a.cpw = pl.cpw[l];
  a.B = pl.batch;
  a.d_in = pl.d_in;
  a.last = l == pl.n_layers - 1;
  a.likelihood = pl.likelihood;
  a.layer = l;
  step_lds(a, lds_floats, nwb, bwd, sd.full_bayes || a.dxw > 0);
  // element-owner prologue: X tile + dF tile <= 512 elements, W/Omega block staged by float4
  const int dpad = round4(a.d);
  a.ws = sd.ws;
  a.fprev_off = l > 0 ? (int)pl.fp_off[l - 1] : 0;
  a.dsrc_off = a.last ? (int)pl.fp_off[l] : (l + 1 < pl.n_layers ? (int)pl.dxp_off[l + 1] : 0);
  // element-owner prologue: up to two elements per thread of the first min(threads, 512); the
  // 4-wave backward also stages its 64-feature W / Omega block by float4 (g, g_{l-1} <= 16), the
  // whole-slice (8-wave) backward and the forward stage nothing there
  const int pro_cap = 2 * min(64 * nwb, 512);
  const bool blk4 = bwd && nwb < 8;
  a.fast = sd.ws != nullptr && TR * (dpad + (bwd ? a.g : 0)) <= pro_cap &&
           (!blk4 || (a.g <= 16 && a.gp <= 16)) && a.R % 4 == 0 && pl.ws_chain < (1 << 29);
  a.xmag = div_magic(dpad);
  a.dmag = div_magic(a.g);
  a.ns = pl.ns[l];
  set_block_map(a, pl.n_row_tiles, pl.n_chains);
  // full_bayesian=True: z rows, hyper partials, per-wave LDS sums [4][round4(2d+1)]
  a.a0 = (l == 0 && pl.a0_off >= 0 && sd.ws) ? sd.ws + pl.a0_off : nullptr;
  a.z = sd.z ? sd.z + pl.omega_off[l] : nullptr;
  a.hp = sd.ws + pl.hpp_off[l];
  a.hpl = sd.ws + pl.hpl_off;
  a.lik_fb = (pl.hyp_flags & DGPRF_HYP_LIK) != 0 && pl.likelihood == DGPRF_LIK_GAUSSIAN;
  // whole-slice staging for the backward (used only where dPhi / dX need W and Omega)
  a.kind_rbf = pl.kind[l] == DGPRF_RBF;
  a.wstage = 0;
  a.wsa_off = a.osa_off = a.osa_st = 0;
  {
    const int nf = 64 * a.cpw, nh = a.kind_rbf ? 2 : 1;
    const int wsa = a.stg_off, osa = wsa + round4(nh * nf * a.g), ost = nf + 4;
    const int end = osa + a.dxw * ost + (sd.full_bayes ? NW * round4(2 * a.d + 1) : 0);
    if (bwd && nwb == 8 && a.cpw % 4 == 0 && a.R % nf == 0 && ((int64_t)a.R * a.g) % 4 == 0 &&
        end <= 38 * 1024) {
      a.wstage = 1;
      a.wsa_off = wsa;
      a.osa_off = osa;
      a.osa_st = ost;
      lds_floats = max(lds_floats, osa + a.dxw * ost);
    }
  }
  a.hred_off = lds_floats;
  if (sd.full_bayes) lds_floats += NW * round4(2 * a.d + 1);
  // whole-slice (8-wave) backward, gW partial tiles of widths that are not a multiple of 16: they
  // leave the MFMA as 16-float row pieces (64 / 56 / 32 B at a row stride of g floats), so they are
  // staged per wave in LDS and the wave's 16 feature rows (contiguous in W) go out as whole 16-byte
  // lanes (config 4, g = 30 / 10).  The 4-wave instances keep dword stores: the staging puts the
  // config-2 backward (168-VGPR budget) 15 VGPRs over (4 spilled without it).
  a.gst_off = 0;
  if (a.wstage && a.g > 1 && (a.g & 15) != 0) {
    if (round4(lds_floats) + nwb * 2 * 16 * a.g <= 40 * 1024) {
      a.gst_off = round4(lds_floats);
      lds_floats = a.gst_off + nwb * 2 * 16 * a.g;
    } else {
      a.wstage = 0;  // no room for the staging next to the slice image: the 4-wave form
    }
  }
  a.a0_sl = 0;
  if (a.a0 && !sd.bd.A1) {  // the A_1 GEMM's K parts (agemm.hip): two slabs, summed here as slab 0 + slab 1
    const int64_t rows = (pl.batch + 31) / 32 * 32;
    if (dgprf::agemm_parts(pl.batch, rows, pl.d_in, pl.d[0], pl.n_rf[0]) == 2)
      a.a0_sl = (int32_t)(rows * pl.n_rf[0]);
  }
  // folded output layer (W-only backward of layer L): W_L [P] then Omega_L rows [d][R + 16] (the
  // padding spreads the 4 k-rows a wave reads over distinct banks), after everything else
  a.rcf = (bwd && a.last && pl.fold_out && !sd.full_bayes && nwb == 4) ? 1 : 0;
  a.rcf_off = 0;
  if (a.rcf) {
    a.rcf_off = round4(lds_floats);
    lds_floats = a.rcf_off + (a.kind_rbf ? 2 : 1) * a.R + a.d * (a.R + 16);
  }
  a.rt_per_rg = 1;
  a.ncw = a.nrw = a.rg_fast = a.gred_off = a.rg_nit = 0;
  a.rw_one = a.cmp = 0;
  a.rw_orows = a.rw_pad = 0;
  a.stamps = nullptr;
  return a;
}

// Row-group backward layout of layer l (floats; xs at 0): false when the layer does not fit it
// (more than 32 chunks per slice, or LDS past 160 KiB).  Shared by dgprf_plan_init (which enables
// the row-group path only when every layer fits) and the launcher.
struct RgCfg {
  int ncw, nrw, nit, fast, aux, red, wsa, osa, ost, hred, gred, total;
};
inline bool rg_config(const dgprf_plan_t& pl, int l, bool fb, RgCfg& c) {
  const int d = pl.d[l], g = pl.n_gp[l], cpw = pl.cpw[l];
  const int dxw = l > 0 ? pl.n_gp[l - 1] : 0;
  const bool rbf = pl.kind[l] == DGPRF_RBF, g1 = g == 1;
  const int NOT = (g + 15) >> 4, CH = 4 * cpw;
  if (CH > 32) return false;
  int ncw = 16;
  while (ncw > CH && ncw > 4) ncw >>= 1;  // largest power of two <= CH
  if (NOT > 2) ncw = 16;                  // wide outputs: no row-waves (their gW sum in LDS)
  c.ncw = ncw;
  c.nrw = 16 / ncw;
  c.nit = (CH + ncw - 1) / ncw;
  if (c.nit > 2) return false;
  const int rows = TR * c.nrw, xst = round4(d) + 1, auxst = g + 1;
  const bool need_x = !(l == 0 && pl.d[0] > 32) || fb;  // layer 0 with A_1 precomputed: no X
  int off = need_x ? round4(rows * xst) : 0;
  c.aux = off;
  off += 2 * round4(rows * auxst);
  c.red = off;
  if (dxw > 0) off += 16 * TR * ((dxw + 15) / 16 * 16);
  const int nf = 64 * cpw;
  c.wsa = off;
  if (fb || dxw > 0) off += round4((rbf ? 2 : 1) * nf * g);
  c.ost = nf + 4;
  c.osa = off;
  off += round4(dxw * c.ost);
  c.hred = off;
  if (fb) off += 16 * round4(2 * d + 1);
  c.gred = off;
  if (c.nrw > 1) off += 16 * (g1 ? c.nit * 2 * 64 : c.nit * NOT * 2 * 256);
  c.total = off;
  c.fast = ((need_x ? rows * round4(d) : 0) + rows * g <= 1024 && pl.ws_chain < (1 << 29)) ? 1 : 0;
  return (int64_t)c.total * 4 <= 160 * 1024;
}

// Large minibatches with one chain: the step's forward is ONE launch of the predictive row / tile
// kernel over all layers (k_forward_rows / k_forward_tiles, every layer's F kept on chip between
// layers) writing complete F_l [B][g_l] into slice 0 of the F partial buffers, instead of L
// feature-sliced launches whose 16 slice partials every consumer re-sums (16x the L2 reads).
// From 8 row tiles per group (B > 1,792): below that the one-tile-per-workgroup forward leaves
// most CUs idle (config 2 at B = 1,024: 59.7 us/step fused vs 48.8 per layer).
inline bool step_fused_fwd(const dgprf_plan_t& pl) {
  return pl.rt_per_group >= 8 && pl.n_chains == 1 && pl.a0_off < 0;
}

// A-tile k-steps of the step kernels for input width d (the KS instance a layer runs)
__host__ __device__ inline int step_ks(int d) { return d <= 4 ? 1 : (d <= 8 ? 2 : (d <= 16 ? 4 : 8)); }

// Output layer folded into its backward ("recompute instead of synchronise"): for a g_L = 1
// Gaussian output layer, every k_step_bwd workgroup of layer L recomputes F_L for its 16 rows over
// all R_L features from the X tile it loads anyway (F_{L-1}), with the layer's whole W_L and
// Omega_L staged in LDS, and forms dF_L (likelihoods/gaussian.py:18-25) in place — so the step has
// no forward launch for layer L and no F_L slice partials.  The recompute is 16x that layer's
// forward work (16 feature slices per row tile), so it is taken only where a launch boundary
// costs more: B <= 256 (per-tile backward), fewer than 4 chains (one feature chunk per wave per
// slice, the chip not full), and at most 128 A-tile k-steps per 4-wave workgroup ((R_L / 16) x
// KS(d_L): config 2's 1,024-feature, d = 8 output layer; not config 3's 2,048 x d = 9, nor config
// 5's 8,192).  W-only steps: a full-Bayes step keeps the forward launch (plan-independent choice
// at enqueue time).  The element-owner prologue must apply (4 waves, d_L <= 28, g_{L-1} <= 16).
inline bool step_fold_out(const dgprf_plan_t& pl) {
#ifdef DGPRF_NO_FOLD  // A/B diagnostic build (scripts/ab_variants.sh), never the product library
  return false;
#endif
  const int L = pl.n_layers - 1;
  const int d = pl.d[L], R = pl.n_rf[L];
  if (pl.rt_per_group != 1 || pl.n_chains >= 4 || pl.n_gp[L] != 1 ||
      pl.likelihood != DGPRF_LIK_GAUSSIAN || (L == 0 && pl.a0_off >= 0) || pl.ws_chain >= (1 << 29))
    return false;
  if (d > 28 || (L > 0 && pl.n_gp[L - 1] > 16) || R % 256 != 0 || (R / 16) * step_ks(d) > 128)
    return false;
  const int P = pl.kind[L] == DGPRF_RBF ? 2 * R : R;
  return (int64_t)(P + d * (R + 16)) * 4 <= 48 * 1024;
}

// Row-wave backward layout of layer l (step_bwdrw_impl.h; floats): false when the layer does not
// fit it — it needs the fused forward's complete F_l (step_fused_fwd), >= 8 row tiles per group,
// d <= 32, g <= 12, 4 or 8 chunks per slice and at most 8 gW accumulator tiles per wave.
struct RwCfg {
  int nch, nwv, wsa, osa, ost, wave0, wstride, hred, gred, total;
  int xst, dst, gpw, orows;  // X / dF tile row strides, W staging row width, staged Omega rows
};
inline bool rw_config(const dgprf_plan_t& pl, int l, bool fb, RwCfg& c, int max_nwv = 16) {
  const int d = pl.d[l], g = pl.n_gp[l], cpw = pl.cpw[l];
  const int dxw = l > 0 ? pl.n_gp[l - 1] : 0;
  const bool rbf = pl.kind[l] == DGPRF_RBF;
  c.nch = 4 * cpw;
  const int nf = 64 * cpw;
  // zero-padded wave tiles and staging, so no fragment read in the chunk body is masked: X rows
  // of 4 KS columns, dF / Y rows of 16 columns, W rows of 4 ceil(g / 4) outputs (1 for g = 1),
  // Omega rows up to 4 KS
  c.xst = 4 * step_ks(d) + 1;
  c.dst = 17;
  c.gpw = g == 1 ? 1 : 4 * ((g + 3) / 4);
  c.orows = 4 * step_ks(d) > d ? 4 * step_ks(d) : d;
  const int xst = c.xst, dst = c.dst;
  if (!step_fused_fwd(pl) || pl.rt_per_group < 8 || d > 32 || g > 12 || dxw > 16 ||
      pl.ws_chain >= (int64_t)1 << 29 ||
      (c.nch != 4 && c.nch != 8) || c.nch * (rbf ? 2 : 1) > 8 || pl.n_rf[l] % nf != 0)
    return false;
  // 16 waves (four per SIMD) when every wave still gets >= 2 row tiles and the layout fits
  // (W-only steps: the full-Bayes body does not fit 128 VGPRs)
  for (c.nwv = pl.rt_per_group >= 32 && max_nwv >= 16 && !fb ? 16 : 8;; c.nwv = 8) {
    int off = 0;
    c.wsa = off;
    if (fb || dxw > 0) off += round4((rbf ? 2 : 1) * nf * c.gpw);
    c.ost = nf + 4;
    c.osa = off;
    off += round4((c.orows > dxw ? c.orows : dxw) * c.ost);
    c.wave0 = off;  // per wave: X tile, dF tile, Y tile, dA transpose scratch [16][20]
    c.wstride = round4(TR * xst) + 2 * round4(TR * dst) + TR * 20;
    off += c.nwv * c.wstride;
    c.hred = off;
    if (fb) off += c.nwv * round4(2 * d + 1);
    c.gred = off;  // 8 slots of gW accumulators
    off += 8 * (g == 1 ? c.nch * 2 * 64 : c.nch * (rbf ? 2 : 1) * 256);
    c.total = off;
    if ((int64_t)c.total * 4 <= 160 * 1024) return true;
    if (c.nwv == 8) return false;
  }
}

// Kernel launch dispatch of the forward / backward over (NOT, G1, RBF, waves) for one A-tile k-step
// count KS (each KS instantiated in its own translation unit, step_fwd_k<KS>.hip / step_bwd_k<KS>.hip).
template <int KS>
void k_step_fwd_launch2(int g, bool rbf, int nw, dim3 grid, size_t lds, hipStream_t s,
                        const LayerK& a);
template <int KS>
void k_step_bwd_launch2(int g, bool rbf, bool fb, bool w8, dim3 grid, size_t lds, hipStream_t s,
                        const LayerK& a);
template <int KS>
void k_step_bwd_rw_launch2(int g, bool rbf, bool fb, bool dx, int nch, int nwv, dim3 grid, size_t lds,
                           hipStream_t s, const LayerK& a);
template <int KS>
void k_step_bwd_rg_launch2(int g, bool rbf, bool fb, int nit, dim3 grid, size_t lds, hipStream_t s,
                           const LayerK& a);

}  // namespace dgprf_sk
