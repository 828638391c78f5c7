// step_kernels.hip — one SGHMC/SGLD step of the DGP-RF sampler on gfx950.
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
#include <cstring>

#include "dgprf_internal.h"

namespace {

constexpr int NW = DGPRF_WAVES;
constexpr int TR = DGPRF_TILE_ROWS;
constexpr int NSM = DGPRF_NS_MAX;
constexpr float LOG_2PI = 1.8378770664093453f;
constexpr int OST = 68;  // LDS row stride of the staged Omega block (16B-aligned rows)

__host__ __device__ __forceinline__ int round4(int x) { return (x + 3) & ~3; }

// Arguments of one forward / backward launch of layer `layer` (host-precomputed).
struct LayerK {
  const float* om;      // Omega_l [d][R] of chain 0 (chain stride om_cs; 0 = shared)
  const float* W;       // W_l [P][g] of chain 0 (chain stride w_cs)
  const float* fprev;   // F_{l-1} partials [NSM][B][gp] of chain 0 (chain stride ws_cs)
  float* fout;          // F_l partials [NSM][B][g]
  const float* dxnext;  // dX_{l+1} partials [NSM][B][g]        (backward, l < L-1)
  float* dxout;         // dX_l partials [NSM][B][dxw]           (backward, l > 0)
  float* gwp;           // gW partials of W_l, row-tile stride w_cs (backward)
  float* logp;          // per-row log p [B]                       (backward, last layer)
  const float* xrows;   // minibatch X rows [B][d_in] (chain stride xrow_cs)
  const float* yrows;   // minibatch Y rows [B][y_cols] (chain stride yrow_cs)
  const float* cptr;    // c_l
  const float* varptr;  // sigma^2
  int64_t w_cs, ws_cs, xrow_cs, yrow_cs, om_cs, der_cs;
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
  // fused SGHMC update (plan.fused_update, W-only steps; models/dgp.py:206-216)
  float* th0;           // theta of chain 0 (chain stride w_cs)
  float* mo0;           // momenta of chain 0 (chain stride w_cs)
  const float* mass;    // [C][L]
  const int64_t* step;
  const float* gwb;     // gW partial rows of chain 0 (ws + gwp_off; row stride w_cs, chain ws_cs)
  unsigned* tick;       // W_1 slice arrival tickets of chain 0 (ws + tick_off, chain stride ws_cs)
  uint64_t seed;
  int32_t pend;         // forward, layer 0: apply the previous step's pending W_1 update first
  int32_t pend_lo;      // w_off of layer 0
  int32_t smap, pad_s;  // slice-major block map (tile_of_block)
  // whole-slice staging (backward, cpw >= 4): the workgroup's W rows [h][64 cpw][g] and Omega rows
  // [dxw][64 cpw + 4] are copied global -> LDS once (global_load_lds) instead of one 64-feature
  // block per chunk with a load round trip and two barriers each
  int32_t wstage, wsa_off, osa_off, osa_st, kind_rbf, pad_w;
  int32_t main_blocks;  // this layer's (row tile, slice) workgroups; extra workgroups follow
  int32_t upd_blocks, upd_layer, upd_lo, upd_hi;  // backward extras: the update of layer upd_layer's
                                                  // W (packed range [upd_lo, upd_hi))
  int32_t gat_blocks, n_layers, upd_t_off, gat_t_off;
  UpdateDev ud;
  BatchDev bd;          // backward extras of the last layer: rows of step t+1 ...
  float* xb_next;       // ... into the other gathered-rows buffer (chain stride ws_cs)
  float* yb_next;
  int32_t yb_cols, pad_f;
};

// Block -> (row tile, slice): blocks are dealt round-robin over the 8 XCDs, so block b's XCD group
// is b % 8; every workgroup of row tile rt gets group rt % 8, so the slice partials it exchanges
// with the neighbouring layers' kernels stay within one L2.  Speed only: correctness never depends
// on placement.  Blocks past the last row tile exit at once.
// Slice-major map (a.smap, the forward applying the pending W_1 update): every row tile of slice sl
// runs on XCD sl % 8 instead, so the 13 workgroups that each sum the slice's gW partials read them
// through one L2.
__device__ __forceinline__ bool tile_of_block(const LayerK& a, int& rt, int& sl) {
  const int b = blockIdx.x, grp = b & 7, idx = b >> 3;
  if (a.smap) {
    const int k = idx / a.n_rt;
    rt = idx - k * a.n_rt;
    sl = grp + 8 * k;
    return sl < a.ns;
  }
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
  const float* gwp;     // gW partials base of chain 0 (chain stride ws_cs, row-tile stride w_total)
  const float* mass;
  const int64_t* step;
  int32_t w_total, n_rt, n_rt_pad, n_layers;
  int32_t lo[DGPRF_MAX_LAYERS], hi[DGPRF_MAX_LAYERS];
  uint64_t seed;
  int64_t ws_cs;
  int32_t step_offset, upd_blocks;
  UpdateDev ud;
  const float* grad_in;
  float* grad_out;
  int64_t grad_cs;      // chain stride of grad_out (w_total, or w_total + hyp_total in full Bayes)
  // gather of step t+1's minibatch rows (graph mode)
  int32_t gather_next, B, d_in, yb_cols;
  BatchDev bd;
  float* xb;
  float* yb;
  // full_bayesian=True: the first hyp_blocks workgroups do the hyper-parameter work
  int32_t hyp_blocks, pad_h;
  HypK hk;
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

__host__ __device__ inline void step_lds(int d, int g, LayerK& a, int& total, int nwb = NW) {
  a.xst = round4(d) + 1;
  a.aux_off = round4(TR * a.xst);
  a.auxst = g + 1;
  a.red_off = a.aux_off + 2 * round4(TR * a.auxst);  // dF tile + Y tile
  // backward: the workgroup's 64-feature block of W_l ([2][64*g] raw) and Omega_l ([64][OST])
  a.stg_off = a.red_off + nwb * TR * 64;  // per-wave reduction rows of nwb waves
  a.os_off = a.stg_off + (2 * 64 * g > 2048 ? round4(2 * 64 * g) : 2048);
  total = a.os_off + 64 * OST;
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
  const bool fromp = inb && (isx ? c < a.gp : true);
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
// The same fragments from the forward's LDS copy of the freshly updated W_1 slice (PEND):
// pw[h][(f - fb0) g + o], nhalf floats per half.
template <int NOT, bool RBF, bool G1>
__device__ __forceinline__ void load_w_frag_lds(const float* pw, int nhalf, int R, int g, int fb0,
                                                int f0, int lr, int lq, float (&wf)[NOT][4][2]) {
#pragma unroll
  for (int ot = 0; ot < NOT; ++ot) {
    const int oc = G1 ? 0 : min(ot * 16 + lr, g - 1);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int fl = min(f0 + 4 * lq + r, R - 1) - fb0;
      wf[ot][r][0] = pw[fl * g + oc];
      wf[ot][r][1] = RBF ? pw[nhalf + fl * g + oc] : 0.f;
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

// ------------------------------------------------------------------------- fused update
// The SGHMC / SGLD update of models/dgp.py:206-216 for W-only steps, run inside the step kernels
// (plan.fused_update): 4 consecutive packed elements e0..e0+3 (e0 % 4 == 0) of chain `chain`.
//   g = W / N + sum_rt gW_rt   (prior N(0,1), models/dgp.py:129-136,171; row-tile partials in order)
//   m <- b m - h N g + sqrt(2 (1 - b) T M) xi,   W <- W + (h / M) m,   h = sqrt(lr / N)
// with the noise xi (and resampled m) the Philox stream (seed, sub = t, purpose, tag = chain) at
// counter quad e0 / 4 — the same values, in the same arithmetic order, as k_step_update.
__device__ __forceinline__ void step_schedule_rt(const UpdateDev& ud, int64_t t, float* lr, float* T,
                                                 int* resample) {
  if (ud.schedule == DGPRF_SCHED_CYCLICAL) step_schedule<true>(ud, t, lr, T, resample);
  else step_schedule<false>(ud, t, lr, T, resample);
}

struct UpdScal {
  float N, h, beta, T;
  int resample;
};
__device__ __forceinline__ UpdScal upd_scalars(const UpdateDev& ud, int64_t t) {
  UpdScal u;
  float lr;
  step_schedule_rt(ud, t, &lr, &u.T, &u.resample);
  u.N = ud.data_size;
  u.h = sqrtf(lr / u.N);
  u.beta = ud.beta;
  return u;
}

__device__ __forceinline__ void sghmc4(const UpdateDev& ud, const UpdScal& u, float M, uint64_t seed,
                                       int64_t t, int chain, int64_t cw, int64_t e0, f4 th, f4 m,
                                       f4 gl, f4* th_new, f4* m_new) {
  const f4 gr = th / u.N + gl;
  const uint32_t quad = (uint32_t)(e0 >> 2);
  if (u.resample) {  // models/dgp.py:209-210 (ignores M, Appendix A.1)
    if (ud.xi_resample) {
      m = *reinterpret_cast<const f4*>(ud.xi_resample + cw + e0);
    } else {
      m = philox_normal4(seed, (uint64_t)t, DGPRF_RNG_RESAMPLE, (uint32_t)chain, quad);
    }
  }
  f4 mn = u.beta * m - (u.h * u.N) * gr;
  const f4 eps = ud.xi ? *reinterpret_cast<const f4*>(ud.xi + cw + e0)
                       : philox_normal4(seed, (uint64_t)t, DGPRF_RNG_NOISE, (uint32_t)chain, quad);
  mn = mn + sqrtf(2.0f * (1.0f - u.beta) * u.T * M) * eps;
  *m_new = mn;
  *th_new = th + (u.h * (1.0f / M)) * mn;
}

// Sum of the row-tile gW partials of element quad e0 (n_rt <= NSM rows, fixed order from row 0;
// rows past n_rt lie outside the descriptor: 0, no memory access).
__device__ __forceinline__ f4 gw_partial_sum(rsrc_t rs, int64_t row_stride, int n_rt, int64_t e0,
                                             bool ok = true) {
  // rows past n_rt (wave-uniform) are not issued at all; masked lanes read 0 without traffic
  f4 v[NSM];
#pragma unroll
  for (int rt = 0; rt < NSM; ++rt)
    v[rt] = rt < n_rt ? bload4(rs, ok ? (uint32_t)((rt * row_stride + e0) * 4) : DGPRF_OOB) : f4zero();
  f4 acc = f4zero();
#pragma unroll
  for (int rt = 0; rt < NSM; ++rt) acc += v[rt];
  return acc;
}

// ------------------------------------------------------------------------- fused update workgroups
// One workgroup's 4 x blockDim packed elements of the update of layer a.upd_layer's W from its
// row-tile gW partials (written by an earlier kernel): extra workgroups of the next layer's
// backward, or the flush kernel.
__device__ __forceinline__ void update_layer_block(const LayerK& a, int j, int chain) {
  const int64_t e0 = a.upd_lo + 4 * ((int64_t)j * blockDim.x + threadIdx.x);
  if (e0 >= a.upd_hi) return;
  const int64_t cw = (int64_t)chain * a.w_cs;
  const f4 th = *reinterpret_cast<const f4*>(a.th0 + cw + e0);
  const f4 m = *reinterpret_cast<const f4*>(a.mo0 + cw + e0);
  const rsrc_t rs = make_rsrc(a.gwb + (int64_t)chain * a.ws_cs, (int64_t)a.n_rt * a.w_cs);
  const f4 gl = gw_partial_sum(rs, a.w_cs, a.n_rt, e0);
  const float M = a.mass[chain * a.n_layers + a.upd_layer];
  // the step counter is read after the parameter and partial loads are in flight
  const int64_t t = *a.step + a.upd_t_off;
  const UpdScal u = upd_scalars(a.ud, t);
  f4 thn, mn;
  sghmc4(a.ud, u, M, a.seed, t, chain, cw, e0, th, m, gl, &thn, &mn);
  if (e0 + 3 < a.upd_hi) {
    st4(a.mo0 + cw + e0, mn);
    st4(a.th0 + cw + e0, thn);
  } else {  // layer padding between align4 offsets stays untouched
    for (int i = 0; i < 4 && e0 + i < a.upd_hi; ++i) {
      a.mo0[cw + e0 + i] = mn[i];
      a.th0[cw + e0 + i] = thn[i];
    }
  }
}

// Extra workgroup j of a backward: the W update first, then the gather of step t+1's rows.
__device__ __forceinline__ void bwd_extra_block(const LayerK& a, int j, int chain) {
  if (j < a.upd_blocks) {
    update_layer_block(a, j, chain);
    return;
  }
  j -= a.upd_blocks;
  const int64_t t = *a.step + a.gat_t_off;
  float* xb = a.xb_next + (int64_t)chain * a.ws_cs;
  float* yb = a.yb_next + (int64_t)chain * a.ws_cs;
  if (a.d_in > GATHER_WIDE) {  // one wave per row
    const int b = j * (int)(blockDim.x >> 6) + (int)(threadIdx.x >> 6);
    if (b < a.B) gather_row_wave(a.bd, a.B, a.d_in, a.yb_cols, xb, yb, chain, t, b, threadIdx.x & 63);
    return;
  }
  const int b = j * (int)blockDim.x + (int)threadIdx.x;
  if (b < a.B) gather_row(a.bd, a.B, a.d_in, a.yb_cols, xb, yb, chain, t, b);
}

__global__ __launch_bounds__(256) void k_layer_update(const LayerK a) {
  update_layer_block(a, (int)blockIdx.x, (int)blockIdx.z);
}

// ------------------------------------------------------------------------- forward
// PEND (layer 0, fused update): the workgroup first applies the previous step's pending update to
// its feature slice of W_1 (both halves: theta, momenta and the 13 row-tile gW partials loaded
// alongside the X tile), keeps the new slice in LDS for its W fragments, and takes an arrival
// ticket; the slice's last workgroup to arrive stores the new theta / momenta at its end — every
// other workgroup of the slice has read the old values by then (its ticket follows its loads), so
// no workgroup can see a half-updated slice.  Every workgroup of the slice computes bit-identical
// values (same inputs, same order, same Philox counters).
template <int KS, int NOT, bool RBF, bool G1, bool PEND, int NWB>
// Minimum waves per SIMD the register allocation must allow.  Single-chain steps run one workgroup
// per CU either way; with C chains per launch (13 x 16 x C workgroups) residency sets throughput:
// the g <= 16, d <= 8 W-only backward at <= 168 VGPRs (3 waves/SIMD) measured 127k -> 156k
// chain-steps/s at C = 64 and single-chain 36.3k -> 36.7k steps/s (config 3's ARC layers +3 %);
// the wider / full-Bayes instances keep their registers (they would spill 20-200 VGPRs; config 5's
// RBF d = 16 layers lost 8 % with 22 spilled).
#ifndef DGPRF_STEP_WPE
#define DGPRF_STEP_WPE 3
#endif
__global__ __launch_bounds__(64 * NWB) void k_step_fwd(const LayerK a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  int rt, sl;
  if (!tile_of_block(a, rt, sl)) return;
  const int chain = blockIdx.z;
  const float* __restrict__ om = a.om + (int64_t)chain * a.om_cs;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, lr = lane & 15, lq = lane >> 4;
  const int R = a.R, g = a.g, d = a.d, B = a.B, cpw = a.cpw;
  const int row0 = rt * TR;
  const int stamp_base = (a.layer * 2) * 4096 + blockIdx.z * gridDim.x + blockIdx.x;
  DGPRF_STAMP(stamp_base, 0);
  float* xs = smem;
  float* red = smem + a.red_off;
  const float* __restrict__ W = a.W + (int64_t)chain * a.w_cs;
  // the slice's 4 cpw 16-feature chunks: iteration i of wave w takes chunk i NWB + w
  auto chunk_f0 = [&](int i) { return ((sl * cpw * 4 + i * NWB) + wave) * 16; };
  const int nit = cpw * 4 / NWB;

  // PEND: old theta / momenta / gW partials of the slice, issued first (up to 4 quads per thread)
  constexpr int PQ = PEND ? 4 : 1;
  const int nfs = 64 * cpw, fb0 = sl * nfs, nhalf = nfs * g;
  const int nvq = max(min(nfs, R - fb0), 0) * g / 4;  // valid quads per half (R g % 4 == 0)
  const int nhq = nhalf / 4, nq = (RBF ? 2 : 1) * nhq;
  const int64_t cw = (int64_t)chain * a.w_cs;
  float* pw = smem + a.stg_off;  // new W_1 slice [h][nhalf]; flag word at pw[8192 / 2]
  f4 pth[PQ], pmo[PQ], pgl[PQ];
  int64_t t_pend = 0;
  if (PEND) {
    t_pend = *a.step;  // the step counter's round trip overlaps the loads below
    const rsrc_t rth = make_rsrc(a.th0 + cw, a.w_cs), rmo = make_rsrc(a.mo0 + cw, a.w_cs);
    const rsrc_t rs = make_rsrc(a.gwb + (int64_t)chain * a.ws_cs, (int64_t)a.n_rt * a.w_cs);
#pragma unroll
    for (int j = 0; j < PQ; ++j) {
      pth[j] = pmo[j] = pgl[j] = f4zero();
      if (256 * j >= nq) continue;  // wave-uniform: nothing issued for empty rounds
      const int q = (int)threadIdx.x + 256 * j, h = q >= nhq ? 1 : 0, ql = q - h * nhq;
      const bool ok = q < nq && ql < nvq;
      const int64_t e0 = a.pend_lo + (int64_t)(h * R + fb0) * g + 4 * ql;
      pth[j] = bload4(rth, ok ? (uint32_t)(e0 * 4) : DGPRF_OOB);
      pmo[j] = bload4(rmo, ok ? (uint32_t)(e0 * 4) : DGPRF_OOB);
      pgl[j] = gw_partial_sum(rs, a.w_cs, a.n_rt, e0, ok);
    }
  }
  // first chunk's fragments: independent of the X tile, issued first
  float omk[8], wf[NOT][4][2];
  if (KS > 0) load_om_frag<KS>(om, R, d, chunk_f0(0), lr, lq, omk);
  if (!PEND) load_w_frag<NOT, RBF, G1>(W, R, g, chunk_f0(0), lr, lq, wf);
  const float cl = a.cptr[(int64_t)chain * a.der_cs];
  DGPRF_STAMP(stamp_base, 1);
  if (a.fast) {
    elem_prologue(a, chain, row0, 0, xs, red, 0, red, red);  // no dF tile: unused targets
  } else if (KS > 0 || !a.a0) {
    load_x_tile(a, chain, row0, xs);
  }
  if (PEND) {
    const int64_t t = t_pend + a.upd_t_off;
    const UpdScal u = upd_scalars(a.ud, t);
    const float M = a.mass[chain * a.n_layers];
#pragma unroll
    for (int j = 0; j < PQ; ++j) {
      const int q = (int)threadIdx.x + 256 * j, h = q >= nhq ? 1 : 0, ql = q - h * nhq;
      if (q < nq) {
        const bool ok = ql < nvq;
        const int64_t e0 = a.pend_lo + (int64_t)(h * R + fb0) * g + 4 * ql;
        f4 thn = f4zero(), mn = f4zero();
        if (ok) sghmc4(a.ud, u, M, a.seed, t, chain, cw, e0, pth[j], pmo[j], pgl[j], &thn, &mn);
        pth[j] = thn;
        pmo[j] = mn;
        *reinterpret_cast<f4*>(pw + h * nhalf + 4 * ql) = thn;  // features >= R stage as zeros
      }
    }
  }
  const float* a0 = KS == 0 && a.a0 ? a.a0 + (int64_t)chain * a.ws_cs + (int64_t)(row0 + lr) * R : nullptr;
  __syncthreads();
  DGPRF_STAMP(stamp_base, 2);
  unsigned ticket = 0u;
  if (PEND) {
    // every thread's old values are in registers (the barrier follows their use): arrive
    if (threadIdx.x == 0) ticket = atomicAdd(a.tick + (int64_t)chain * a.ws_cs + 32 * sl, 1u);
    load_w_frag_lds<NOT, RBF, G1>(pw, nhalf, R, g, fb0, chunk_f0(0), lr, lq, wf);
  }

  float xf[8];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) xf[ks] = (ks < KS && 4 * ks < d) ? xs[lr * a.xst + 4 * ks + lq] : 0.f;

  f4 acc[NOT], acs[NOT];
#pragma unroll
  for (int ot = 0; ot < NOT; ++ot) acc[ot] = acs[ot] = f4zero();
  float acc1 = 0.f;  // G1: per-lane partial of F[row lr]
  DGPRF_STAMP(stamp_base, 6);
  for (int i = 0; i < nit; ++i) {
    const int f0 = chunk_f0(i);
    if (f0 >= R) break;
    const f4 at = (KS == 0 && a0) ? *reinterpret_cast<const f4*>(a0 + f0 + 4 * lq)
                                  : a_tile<KS, false>(om, R, d, f0, omk, xf, xs, a.xst, lr, lq);
    float p0[4], p1[4];
    features<RBF>(at, cl, p0, p1);
    float wc[NOT][4][2];
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool ok = w_ok<G1>(ot, r, R, g, f0, lr, lq);
        wc[ot][r][0] = keep(wf[ot][r][0], ok);
        wc[ot][r][1] = keep(wf[ot][r][1], ok);
      }
    if (i + 1 < nit) {  // prefetch the next chunk (clamped loads are always in range)
      if (KS > 0) load_om_frag<KS>(om, R, d, chunk_f0(i + 1), lr, lq, omk);
      if (PEND) load_w_frag_lds<NOT, RBF, G1>(pw, nhalf, R, g, fb0, chunk_f0(i + 1), lr, lq, wf);
      else load_w_frag<NOT, RBF, G1>(W, R, g, chunk_f0(i + 1), lr, lq, wf);
    }
    if (G1) {
      // g == 1: F[row lr] += sum_f Phi[lr][f] W[f], 4 features per lane (VALU)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        acc1 = fmaf(p0[r], wc[0][r][0], acc1);
        if (RBF) acc1 = fmaf(p1[r], wc[0][r][1], acc1);
      }
    } else {
#pragma unroll
      for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          acc[ot] = mfma16(wc[ot][r][0], p0[r], acc[ot]);
          if (RBF) acs[ot] = mfma16(wc[ot][r][1], p1[r], acs[ot]);
        }
    }
  }
  DGPRF_STAMP(stamp_base, 7);
  // acc[ot][r] = F[row lr][ot*16 + 4lq + r]; sum the 4 waves' feature chunks in LDS.
  constexpr int GP = NOT * 16;
  float* redw = red + wave * TR * GP;
  if (G1) {
    acc1 += __shfl_xor(acc1, 16);
    acc1 += __shfl_xor(acc1, 32);
    if (lq == 0) redw[lr * GP] = acc1;
  } else {
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
      for (int r = 0; r < 4; ++r) redw[lr * GP + ot * 16 + 4 * lq + r] = acc[ot][r] + acs[ot][r];
  }
  DGPRF_STAMP(stamp_base, 3);
  if (PEND && threadIdx.x == 0) pw[4096] = ticket == (unsigned)a.n_rt - 1u ? 1.f : 0.f;
  __syncthreads();
  float* fp = a.fout + (int64_t)chain * a.ws_cs + (int64_t)sl * B * g;
  for (int e = threadIdx.x; e < TR * g; e += blockDim.x) {
    const int r = e / g, o = e - r * g, b = row0 + r;
    if (b < B) {
      float v = red[r * GP + o];
#pragma unroll
      for (int w = 1; w < NWB; ++w) v += red[w * TR * GP + r * GP + o];
      fp[(int64_t)b * g + o] = v;
    }
  }
  if (PEND && pw[4096] != 0.f) {  // the slice's last arrival: store the new W_1 slice
#pragma unroll
    for (int j = 0; j < PQ; ++j) {
      const int q = (int)threadIdx.x + 256 * j, h = q >= nhq ? 1 : 0, ql = q - h * nhq;
      if (q < nq && ql < nvq) {
        const int64_t e0 = a.pend_lo + (int64_t)(h * R + fb0) * g + 4 * ql;
        st4(a.mo0 + cw + e0, pmo[j]);
        st4(a.th0 + cw + e0, pth[j]);
      }
    }
    if (threadIdx.x == 0) atomicExch(a.tick + (int64_t)chain * a.ws_cs + 32 * sl, 0u);  // next launch
  }
#ifdef DGPRF_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  DGPRF_STAMP(stamp_base, 14);
}

// ------------------------------------------------------------------------- backward
// Whole-slice staging (a.wstage): W rows [fb0, fb0 + 64 cpw) of both halves (contiguous runs of
// 64 cpw g floats in W) and Omega rows k < dxw over the same features (runs of 64 cpw floats, one
// LDS row of 64 cpw + 4 each) as 16-byte global_load_lds: lane-linear LDS destinations, no VGPRs,
// every copy in flight at once; the prologue's barrier waits for them.  The slice lies inside the
// layer (R % (64 cpw) == 0) and every run starts 16-byte aligned (R g % 4 == 0).
__device__ __forceinline__ void stage_slice_lds(const LayerK& a, const float* W, const float* om,
                                                int fb0, float* smem) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nf = 64 * a.cpw, g = a.g, R = a.R;
  const int n4 = nf * g / 4;  // float4 per half
  const int nh = a.kind_rbf ? 2 : 1;
  for (int h = 0; h < nh; ++h) {
    const float* src = W + ((int64_t)h * R + fb0) * g;
    float* dst = smem + a.wsa_off + h * nf * g;
    for (int i0 = wave * 64; i0 < n4; i0 += (int)blockDim.x) {
      if (i0 + lane < n4)
        __builtin_amdgcn_global_load_lds(src + 4 * (i0 + lane), dst + 4 * i0, 16, 0, 0);
    }
  }
  const int per_row = nf / 256;  // 256-float instructions per Omega row (cpw >= 4)
  for (int j = wave; j < a.dxw * per_row; j += (int)(blockDim.x >> 6)) {
    const int k = j / per_row, c = j - k * per_row;
    __builtin_amdgcn_global_load_lds(om + (int64_t)k * R + fb0 + c * 256 + 4 * lane,
                                     smem + a.osa_off + k * a.osa_st + c * 256, 16, 0, 0);
  }
}


// NWB: waves per workgroup (8: W-only, whole-slice LDS image); FUSED: the fused update's extra
// workgroups (own instantiations, so their registers never burden the plain kernels).
template <int KS, int NOT, bool RBF, bool G1, bool FB, int NWB, bool FUSED>
__global__ __launch_bounds__(64 * NWB) __attribute__((amdgpu_waves_per_eu((NOT == 1 && !FB && (KS == 1 || KS == 2 || (KS == 4 && !RBF))) ? DGPRF_STEP_WPE : 1))) void k_step_bwd(const LayerK a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  if (FUSED && (int)blockIdx.x >= a.main_blocks) {  // fused update of W_{l+2} / next-batch gather
    bwd_extra_block(a, (int)blockIdx.x - a.main_blocks, (int)blockIdx.z);
    return;
  }
  constexpr bool WST = NWB == 8;  // whole-slice staging (a.wstage == 1 exactly then)
  int rt, sl;
  if (!tile_of_block(a, rt, sl)) return;
  const int chain = blockIdx.z;
  const float* __restrict__ om = a.om + (int64_t)chain * a.om_cs;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, lr = lane & 15, lq = lane >> 4;
  const int R = a.R, g = a.g, d = a.d, B = a.B, cpw = a.cpw, dxw = a.dxw;
  const int row0 = rt * TR;
  const int stamp_base = (a.layer * 2 + 1) * 4096 + blockIdx.z * gridDim.x + blockIdx.x;
  DGPRF_STAMP(stamp_base, 0);
  float* xs = smem;
  float* dfs = smem + a.aux_off;
  const int dfst = a.auxst;
  float* red = smem + a.red_off;
  const float* __restrict__ W = a.W + (int64_t)chain * a.w_cs;
  // iteration i of wave w takes chunk i NWB + w of the slice (8-wave workgroups: whole-slice
  // staging only, a.wstage)
  auto chunk_f0 = [&](int i) { return ((sl * cpw * 4 + i * NWB) + wave) * 16; };
  const int nit = cpw * 4 / NWB;
  constexpr int KGM = 4 * NOT;  // k-steps of the dPhi contraction (K = g)
  const int ND = (dxw + 15) >> 4;
  // dPhi / dA are needed for dX (l > 0) and, with full_bayesian=True, for every layer
  const bool dphi = FB || dxw > 0;

  // first chunk's fragments, issued before the dependent partial sums
  float omk[8];
  if (KS > 0) load_om_frag<KS>(om, R, d, chunk_f0(0), lr, lq, omk);
  // full_bayesian=True: z fragments of the Dz = dA z^T tiles (d <= 32 when KS > 0: two 16-dim
  // tiles prefetched with the Omega fragments; wider layers load them in the chunk loop)
  constexpr int NZ = KS > 0 ? (4 * KS + 15) / 16 : 0;
  const rsrc_t rz = make_rsrc(a.z, FB ? (int64_t)d * R : 0);
  auto z_frag = [&](int f0, int dt) -> f4 {
    const int k = dt * 16 + lr;
    return bload4(rz, k < d && f0 + 4 * lq < R ? (uint32_t)(((int64_t)k * R + f0 + 4 * lq) * 4)
                                               : DGPRF_OOB);
  };
  f4 zpf[NZ > 0 ? NZ : 1];
  if (FB)
#pragma unroll
    for (int dt = 0; dt < NZ; ++dt) zpf[dt] = z_frag(chunk_f0(0), dt);
  // dPhi / dX A operands (W_l rows and Omega_l rows of this workgroup's 64-feature block) are
  // staged through LDS as W [2][64*g] (raw rows) and Omega [rows][OST]; the fragment reads zero
  // feature rows >= R.
  float* wsl = smem + a.stg_off;
  float* osl = smem + a.os_off;
  const int nwh = 64 * g, nwt = RBF ? 2 * nwh : nwh, nom = dxw * 64;
  // general path: clamped scalar loads (contiguous runs), used when a.fast == 0 and for cpw > 1
  constexpr int NJW = 8 * NOT;  // >= 2*64*g/256
  constexpr int NJO = 16;       // >= 64*64/256
  float stw[NJW], sto[NJO];
  auto stage_load = [&](int fb) {
    const int64_t rg = (int64_t)R * g;
#pragma unroll
    for (int j = 0; j < NJW; ++j) {
      const int e = min((int)threadIdx.x + 256 * j, nwt - 1);
      const int h = e >= nwh, e2 = e - h * nwh;
      stw[j] = W[h * rg + min((int64_t)fb * g + e2, rg - 1)];
    }
#pragma unroll
    for (int j = 0; j < NJO; ++j) {
      const int e = min((int)threadIdx.x + 256 * j, max(nom - 1, 0));
      sto[j] = om[(int64_t)(e >> 6) * R + min(fb + (e & 63), R - 1)];
    }
  };
  auto stage_store = [&](int fb) {
#pragma unroll
    for (int j = 0; j < NJW; ++j) {
      const int e = (int)threadIdx.x + 256 * j;
      if (e < nwt) wsl[e] = stw[j];
    }
#pragma unroll
    for (int j = 0; j < NJO; ++j) {
      const int e = (int)threadIdx.x + 256 * j;
      if (e < nom) osl[(e >> 6) * OST + (e & 63)] = fb + (e & 63) < R ? sto[j] : 0.f;
    }
  };
  const int fb0 = (sl * cpw) * 64;
  const float cl = a.cptr[(int64_t)chain * a.der_cs];
  const float* fpl = a.fout + (int64_t)chain * a.ws_cs;        // F_L partials (last layer)
  const float* dxn = a.dxnext + (int64_t)chain * a.ws_cs;      // dX_{l+1} partials
  const float* yr = a.yrows + (int64_t)chain * a.yrow_cs;
  float* ysh = dfs + round4(TR * dfst);
  const int yc = a.likelihood == DGPRF_LIK_GAUSSIAN ? g : 1;
  if (a.fast) {
    // ---- single burst: W/Omega block, X tile, dF (or F_L) partials and Y rows
    f4 sw[2], so;
    if (WST && dphi) stage_slice_lds(a, W, om, fb0, smem);
    if (!WST && dphi) {
      const rsrc_t rw = make_rsrc(W, (int64_t)(RBF ? 2 : 1) * R * g);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int i = (int)threadIdx.x + 256 * j, h = i >= 16 * g, q = i - h * 16 * g;
        const uint32_t off = (uint32_t)((((h * R) + fb0) * g + 4 * q) * 4);
        sw[j] = bload4(rw, i < (RBF ? 32 : 16) * g ? off : DGPRF_OOB);
      }
      const rsrc_t ro = make_rsrc(om, (int64_t)dxw * R);
      const int k = threadIdx.x >> 4, c4 = threadIdx.x & 15;
      so = bload4(ro, k < dxw && fb0 + 4 * c4 < R ? (uint32_t)((k * R + fb0 + 4 * c4) * 4) : DGPRF_OOB);
    }
    DGPRF_STAMP(stamp_base, 1);
    elem_prologue(a, chain, row0, TR * g, xs, dfs, dfst, ysh, red);
    if (!WST && dphi) {
#pragma unroll
      for (int j = 0; j < 2; ++j) *reinterpret_cast<f4*>(wsl + 4 * ((int)threadIdx.x + 256 * j)) = sw[j];
      *reinterpret_cast<f4*>(osl + (threadIdx.x >> 4) * OST + 4 * (threadIdx.x & 15)) = so;
    }
    DGPRF_STAMP(stamp_base, 4);
  } else {
    if (WST && dphi) stage_slice_lds(a, W, om, fb0, smem);
    if (!WST && dphi) stage_load(fb0);
    if (KS > 0 || !a.a0 || FB) load_x_tile(a, chain, row0, xs);
    for (int e = threadIdx.x; e < TR * g; e += blockDim.x) {  // dF (or F_L) slice sums; Y alongside
      const int r = e / g, o = e - r * g, b = row0 + r, bc = min(b, B - 1);
      const float v = sum_slices((a.last ? fpl : dxn) + (int64_t)bc * g + o, (int64_t)B * g);
      dfs[r * dfst + o] = b < B ? v : 0.f;
      if (a.last) ysh[r * dfst + o] = yr[(int64_t)bc * a.y_cols + min(o, yc - 1)];
    }
  }

  // dF_l tile [16][g]: the last layer turns F_L into the likelihood gradient in place;
  // otherwise dF_l = dX_{l+1}[:, :g_l] (already summed above)
  if (a.last) {
    // likelihood gradient dF = -(1/B) dlogp/dF (likelihoods/gaussian.py:18-25, softmax.py:8-15)
    __syncthreads();
    if (threadIdx.x < TR) {
      const int r = threadIdx.x, b = row0 + r;
      float* df = dfs + r * dfst;
      float lvrow = 0.f;
      if (b < B) {
        const float* y = ysh + r * dfst;
        const float invB = 1.0f / (float)B;
        float logp = 0.f;
        if (a.likelihood == DGPRF_LIK_GAUSSIAN) {
          const float var = a.varptr[(int64_t)chain * a.der_cs];
          const float logvar = logf(var);
          float lv = 0.f;  // d(-log p)/d lik_log_var = sum_o (1 - diff^2/var)/2
          for (int o = 0; o < g; ++o) {
            const float diff = y[o] - df[o];
            logp += -0.5f * (LOG_2PI + logvar + diff * diff / var);
            df[o] = -(diff / var) * invB;
            lv += 0.5f * (1.f - diff * diff / var);
          }
          lvrow = lv * invB;
        } else {
          float mx = -INFINITY;
          for (int o = 0; o < g; ++o) mx = fmaxf(mx, df[o]);
          float se = 0.f;
          for (int o = 0; o < g; ++o) se += expf(df[o] - mx);
          const float lse = mx + logf(se);
          // int32(Y[:, 0]) (likelihoods/softmax.py:14); a label outside [0, g) poisons log p and
          // the gradient with NaN instead of scoring a clamped class (TF raises on it)
          const int label = (int)y[0];
          const float bad = (label >= 0 && label < g) ? 0.f : __builtin_nanf("");
          for (int o = 0; o < g; ++o) {
            const float f = df[o];
            if (o == label) logp = f - lse;
            df[o] = (expf(f - lse) - (o == label ? 1.f : 0.f)) * invB + bad;
          }
          logp += bad;
        }
        if (sl == 0) a.logp[(int64_t)chain * a.ws_cs + b] = logp;
      }
      if (FB && a.lik_fb) {  // the row tile's lik_log_var partial (lanes 0..15, fixed order)
        const float v = sum16(lvrow);
        if (r == 0 && sl == 0) a.hpl[(int64_t)chain * a.ws_cs + rt] = v;
      }
    }
  }
  if (!WST && !a.fast && dphi) stage_store(fb0);
  __syncthreads();
  DGPRF_STAMP(stamp_base, 2);

  float xf[8];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) xf[ks] = (ks < KS && 4 * ks < d) ? xs[lr * a.xst + 4 * ks + lq] : 0.f;
  // dF fragments: dff[ks] = dF[row lr][4ks+lq]        (B operand of dPhi, K = g)
  //               dfg[ot][r] = dF[row 4lq+r][ot*16+lr] (B operand of gW, K = rows)
  float dff[KGM];
#pragma unroll
  for (int ks = 0; ks < KGM; ++ks) {
    const int o = 4 * ks + lq;
    dff[ks] = (o < g) ? dfs[lr * dfst + o] : 0.f;
  }
  float dfg[NOT][4];
#pragma unroll
  for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int o = ot * 16 + lr;
      dfg[ot][r] = (o < g) ? dfs[(4 * lq + r) * dfst + o] : 0.f;
    }
  const int KG = (g + 3) >> 2;
  // g == 1 operands: dF[row lr] and dF[rows 4lq..4lq+3] in every lane
  const float dg1 = G1 ? dfs[lr * dfst] : 0.f;
  float dg4[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) dg4[r] = G1 ? dfs[(4 * lq + r) * dfst] : 0.f;

  float* gwp = a.gwp + (int64_t)chain * a.ws_cs + (int64_t)rt * a.w_cs;
  f4 dxa[4] = {f4zero(), f4zero(), f4zero(), f4zero()};
  // full_bayesian=True: per-wave sums over this row tile and the wave's features of
  //   hw[k]     = sum_b X[b][k] (dA z^T)[b][k]   (-> log_inv_ls)
  //   hw[d + k] = sum_b X[b][k] rowsum(dA)[b]    (-> mean)
  //   hw[2d]    = sum dPhi * Phi                  (-> log_amp)
  const int hst = round4(2 * d + 1);
  float* hw = smem + a.hred_off + wave * hst;
  float ampl = 0.f;
  if (FB)
    for (int e = lane; e < hst; e += 64) hw[e] = 0.f;
  for (int i = 0; i < nit; ++i) {
    const int f0 = chunk_f0(i);
    if (f0 >= R) break;
    if (i > 0) {
      if (KS > 0) load_om_frag<KS>(om, R, d, f0, lr, lq, omk);
      if (FB)
#pragma unroll
        for (int dt = 0; dt < NZ; ++dt) zpf[dt] = z_frag(f0, dt);
      if (!WST && dphi) {
        stage_load((sl * cpw + i) * 64);
        __syncthreads();  // every wave is done with the previous block
        stage_store((sl * cpw + i) * 64);
        __syncthreads();
      }
    }
    // ---- phase 1: LDS operands, both A-tile orientations and dPhi (independent chains)
    //   at_t: rows in registers  (gW = Phi^T dF,   K = rows)
    //   at_n: features in registers (dA -> dX = dA Omega^T, K = features)
    //   dPhi = dF W^T in the features-in-registers orientation (K = g)
    float wd0[KGM], wd1[KGM];
    f4 oxv[4];
    // this chunk's 64-feature block: the per-chunk staging buffers, or its rows of the slice image
    const float* wsc = WST ? smem + a.wsa_off + i * NWB * 16 * g : wsl;
    const int whalf = WST ? 64 * cpw * g : nwh;
    const float* osc = WST ? smem + a.osa_off + i * NWB * 16 : osl;
    const int ostc = WST ? a.osa_st : OST;
    if (dphi) {
      const bool frow = f0 + lr < R;
#pragma unroll
      for (int ks = 0; ks < KGM; ++ks) {
        const int o = 4 * ks + lq, wo = (wave * 16 + lr) * g + o;
        const bool ok = o < g && frow;
        wd0[ks] = G1 ? 0.f : (ok ? wsc[wo] : 0.f);
        wd1[ks] = (G1 || !RBF) ? 0.f : (ok ? wsc[whalf + wo] : 0.f);
      }
      // rows k >= dxw of the staged block are never written: they only feed discarded outputs
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        oxv[dt] = *reinterpret_cast<const f4*>(osc + (dt * 16 + lr) * ostc + wave * 16 + 4 * lq);
    }
    // layer 0 with d > 32: both orientations read the precomputed A_1 (k_step_agemm)
    const float* a0 = KS == 0 && a.a0 ? a.a0 + (int64_t)chain * a.ws_cs + (int64_t)row0 * R + f0
                                      : nullptr;
    f4 at_t;
    if (KS == 0 && a0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) at_t[r] = a0[(int64_t)(4 * lq + r) * R + lr];
    } else {
      at_t = a_tile<KS, true>(om, R, d, f0, omk, xf, xs, a.xst, lr, lq);
    }
    f4 at_n = f4zero(), dpc = f4zero(), dps = f4zero();
    if (dphi) {
      at_n = (KS == 0 && a0) ? *reinterpret_cast<const f4*>(a0 + (int64_t)lr * R + 4 * lq)
                             : a_tile<KS, false>(om, R, d, f0, omk, xf, xs, a.xst, lr, lq);
      if (G1) {
        // g == 1: dPhi[b][f] = dF[b] W[f] (outer product, VALU)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int fl = wave * 16 + 4 * lq + r;
          const bool ok = f0 + 4 * lq + r < R;
          dpc[r] = ok ? dg1 * wsc[fl] : 0.f;
          dps[r] = (ok && RBF) ? dg1 * wsc[whalf + fl] : 0.f;
        }
      } else {
#pragma unroll
        for (int ks = 0; ks < KGM; ++ks) {
          if (ks < KG) {
            dpc = mfma16(wd0[ks], dff[ks], dpc);
            if (RBF) dps = mfma16(wd1[ks], dff[ks], dps);
          }
        }
      }
    }
    // ---- phase 2: transcendentals of both tiles, batched
    float q0[4], q1[4];
    features<RBF>(at_t, cl, q0, q1);
    float da[4];
    if (dphi) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (RBF) {
          float sv, cv;
          rf_sincos(at_n[r], &sv, &cv);
          da[r] = -(cl * sv) * dpc[r] + (cl * cv) * dps[r];
          if (FB) ampl += dpc[r] * (cl * cv) + dps[r] * (cl * sv);
        } else {
          da[r] = at_n[r] > 0.f ? cl * dpc[r] : 0.f;
          if (FB) ampl += dpc[r] * (cl * fmaxf(at_n[r], 0.f));
        }
      }
    }
    DGPRF_STAMP(stamp_base, 8);
    // ---- phase 3: gW_l partial of this row tile, then dX
    if (G1) {
      // g == 1: gW[f] = sum_b Phi[b][f] dF[b]: 4 rows per lane, then across the 4 row groups
      float gc = 0.f, gs = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        gc = fmaf(q0[r], dg4[r], gc);
        if (RBF) gs = fmaf(q1[r], dg4[r], gs);
      }
      gc += __shfl_xor(gc, 16);
      gc += __shfl_xor(gc, 32);
      if (RBF) {
        gs += __shfl_xor(gs, 16);
        gs += __shfl_xor(gs, 32);
      }
      const int f = f0 + lr;
      if (lq == 0 && f < R) {
        gwp[f] = gc;
        if (RBF) gwp[R + f] = gs;
      }
    } else {
#pragma unroll
      for (int ot = 0; ot < NOT; ++ot) {
        f4 gc = f4zero(), gs = f4zero();
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          gc = mfma16(q0[r], dfg[ot][r], gc);
          if (RBF) gs = mfma16(q1[r], dfg[ot][r], gs);
        }
        DGPRF_STAMP(stamp_base, 9);
        // gc[r] = gW[f0 + 4lq + r][ot*16 + lr]
        const int o = ot * 16 + lr;
        if (o < g) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int f = f0 + 4 * lq + r;
            if (f < R) {
              gwp[(int64_t)f * g + o] = gc[r];
              if (RBF) gwp[(int64_t)(R + f) * g + o] = gs[r];
            }
          }
        }
      }
    }
    DGPRF_STAMP(stamp_base, 6);
    if (dxw > 0) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        if (dt < ND) {
#pragma unroll
          for (int r = 0; r < 4; ++r) dxa[dt] = mfma16(oxv[dt][r], da[r], dxa[dt]);
        }
    }
    if (FB) {
      // rowsum(dA) over this chunk: the lane's 4 features, then the 4 feature groups
      float rs = (da[0] + da[1]) + (da[2] + da[3]);
      rs += __shfl_xor(rs, 16);
      rs += __shfl_xor(rs, 32);
      // Dz = dA z^T in 16-dim tiles of the layer input (same contraction as dX with z rows),
      // contracted with the X tile over the 16 rows right away (linear in the features)
      for (int dt = 0; dt * 16 < d; ++dt) {
        f4 zf;
        if (NZ > 0) {
          zf = zpf[0];
#pragma unroll
          for (int q = 1; q < NZ; ++q)
            if (dt == q) zf = zpf[q];
        } else {
          zf = z_frag(f0, dt);
        }
        f4 dz = f4zero();
#pragma unroll
        for (int r = 0; r < 4; ++r) dz = mfma16(zf[r], da[r], dz);
        // dz[r] = Dz[row lr][dt*16 + 4lq + r]
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int kk = dt * 16 + 4 * lq + r;
          const float xv = kk < d ? xs[lr * a.xst + kk] : 0.f;
          const float s1 = sum16(xv * dz[r]);
          const float s2 = sum16(xv * rs);
          if (lr == 0 && kk < d) {
            hw[kk] += s1;
            hw[d + kk] += s2;
          }
        }
      }
    }
  }
  DGPRF_STAMP(stamp_base, 3);
  if (FB) {
    // log_amp term over the wave, then the workgroup's partial row [2d+1] in wave order
    float v = sum16(ampl);
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    if (lane == 0) hw[2 * d] = v;
    __syncthreads();
    float* hp = a.hp + (int64_t)chain * a.ws_cs + ((int64_t)rt * NSM + sl) * hst;
    const float* h0 = smem + a.hred_off;
    for (int e = threadIdx.x; e < 2 * d + 1; e += blockDim.x)
      hp[e] = ((h0[e] + h0[hst + e]) + h0[2 * hst + e]) + h0[3 * hst + e];  // FB: NWB == 4
  }
  if (dxw > 0) {
    // dxa[dt][r] = dX[row lr][dt*16 + 4lq + r]; sum the 4 waves in LDS, store the slice partial.
    const int DP = ND * 16;
    float* redw = red + wave * TR * DP;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
      if (dt < ND)
#pragma unroll
        for (int r = 0; r < 4; ++r) redw[lr * DP + dt * 16 + 4 * lq + r] = dxa[dt][r];
    __syncthreads();
    float* dxp = a.dxout + (int64_t)chain * a.ws_cs + (int64_t)sl * B * dxw;
    for (int e = threadIdx.x; e < TR * dxw; e += blockDim.x) {
      const int r = e / dxw, k = e - r * dxw, b = row0 + r;
      if (b < B) {
        float v = red[r * DP + k];
#pragma unroll
        for (int w = 1; w < NWB; ++w) v += red[w * TR * DP + r * DP + k];
        dxp[(int64_t)b * dxw + k] = v;
      }
    }
  }
#ifdef DGPRF_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  DGPRF_STAMP(stamp_base, 14);
}

struct GatherK {
  BatchDev bd;
  const int64_t* step;
  float* xb;  // chain 0 (chain stride ws_cs)
  float* yb;
  int64_t ws_cs;
  int32_t B, d_in, yb_cols, step_offset;
};

__global__ void k_gather(const GatherK a) {
  const int chain = blockIdx.y;
  const int64_t t = *a.step + a.step_offset;
  if (a.d_in > GATHER_WIDE) {  // one wave per row
    const int b = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (b < a.B)
      gather_row_wave(a.bd, a.B, a.d_in, a.yb_cols, a.xb + (int64_t)chain * a.ws_cs,
                      a.yb + (int64_t)chain * a.ws_cs, chain, t, b, threadIdx.x & 63);
    return;
  }
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= a.B) return;
  gather_row(a.bd, a.B, a.d_in, a.yb_cols, a.xb + (int64_t)chain * a.ws_cs,
             a.yb + (int64_t)chain * a.ws_cs, chain, t, b);
}

// Two N(0,1) of counter quad `quad`: words (0,1) (half 0) or (2,3) (half 1) — the same values
// philox_normal4 returns in lanes 2*half, 2*half+1.
__device__ __forceinline__ void philox_normal2(uint64_t seed, uint64_t sub, uint32_t purpose,
                                               uint32_t tag, uint32_t quad, int half, float* z0,
                                               float* z1) {
  u32x4 c;
  c.x = quad;
  c.y = (uint32_t)sub;
  c.z = (uint32_t)(sub >> 32);
  c.w = (purpose << 24) | (tag & 0x00FFFFFFu);
  const u32x4 r = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  box_muller(half ? r.z : r.x, half ? r.w : r.y, z0, z1);
}

typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 ld2(const float* p) { return *reinterpret_cast<const f2*>(p); }
__device__ __forceinline__ void st2(float* p, f2 v) { *reinterpret_cast<f2*>(p) = v; }

// One wave per workgroup, four parameters per lane: the gW partial sums (16 row tiles x 16 bytes
// per lane) are spread over many workgroups instead of concentrated on a few CUs; row tiles
// past n_row_tiles and lanes past w_total lie outside the buffer descriptors (zero, no memory
// traffic), so every load is issued before the first branch.  Specialised on the rarely-used
// paths: GIN (gradient supplied), GONLY (gradient only), XI (injected noise), CYC (cyclical).
constexpr int UPD_THREADS = 64;
__device__ __forceinline__ f2 bload2(rsrc_t r, uint32_t byte_off) {
  return __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(r, byte_off, 0, 0));
}

// One N(0,1) of the hyper-parameter streams (not inlined: the hyper path runs once per step on
// a few CUs, where instruction-cache misses, not arithmetic, set its duration).
__device__ __noinline__ float normal_at(uint64_t seed, uint64_t t, uint32_t purpose, uint32_t chain,
                                        int64_t slot) {
  const f4 z = philox_normal4(seed, t, purpose, chain, (uint32_t)(slot >> 2));
  return z[slot & 3];
}

// Omega elements rebuilt per hyper workgroup (16 per lane)
constexpr int HYP_EPB = UPD_THREADS * 16;

// One hyper workgroup (full_bayesian=True).  The backward left per-workgroup partials
//   [n_rt][NSM][hs]: sum_b X[b][k](dA z^T)[b][k] (k < d), sum_b X[b][k] rowsum(dA)[b], sum dPhi*Phi
// and per row tile the Gaussian lik_log_var term.  Every workgroup of layer l reduces them in the
// same fixed order, forms
//   g_log_amp = sum dPhi*Phi + log_amp/N,   g_lis[k] = exp(lis[k]) sum(...)[k] + lis[k]/N
//   (scalar lis: summed over k),            g_mean[k] = sum_b X[b][k] rowsum(dA)[b] + mean[k]/N
// and applies the SGHMC update of models/dgp.py:206-216 (own momentum, mass and Philox stream) to
// identical new values in LDS; it then rebuilds its HYP_EPB elements of
// Omega_l = exp(lis)[:,None] z_l + mean[:,None] (kernels/RBF.py:43-53, layers/rf_layers.py:34-38).
// The last workgroup of the layer to finish reading the old values (arrival counter, no waiting)
// stores the new hyp / hmom, so no workgroup can read a half-updated set.  Gradient-only mode
// writes dU/d(hyper) into grad_out instead (one workgroup per layer, nothing rebuilt).
template <bool GONLY, bool XI, bool CYC>
__device__ void hyper_block(const UpdK& a, int hb, int chain, float* sm, int sb) {
  const HypK& k = a.hk;
  const int tid = threadIdx.x, L = a.n_layers;
  constexpr int NT = UPD_THREADS;
  float* hyp = k.hyp + (int64_t)chain * k.hyp_cs;
  float* hm = k.hmom + (int64_t)chain * k.hyp_total;
  const float* hmass = k.hmass + chain * DGPRF_HMASS;
  float* gout = a.grad_out + (int64_t)chain * a.grad_cs + a.w_total;
  const UpdateDev& ud = a.ud;
  const float N = ud.data_size;
  const int64_t t = *a.step + (int64_t)a.step_offset;
  float lr, T;
  int resample;
  step_schedule<CYC>(ud, t, &lr, &T, &resample);
  const float h = sqrtf(lr / N), beta = ud.beta;
  // SGHMC update of hyper slot `slot` (value v, momentum m, mass slot midx); returns the new value
  auto upd = [&](int64_t slot, float g, float v, float m, int midx, float* m_out) -> float {
    if (GONLY) {
      gout[slot] = g;
      return v;
    }
    const float M = hmass[midx];
    if (resample)
      m = (XI && ud.xi_hyp_resample)
              ? ud.xi_hyp_resample[(int64_t)chain * k.hyp_total + slot]
              : normal_at(a.seed, (uint64_t)t, DGPRF_RNG_HYPER_RESAMPLE, chain, slot);
    const float eps = (XI && ud.xi_hyp) ? ud.xi_hyp[(int64_t)chain * k.hyp_total + slot]
                                        : normal_at(a.seed, (uint64_t)t, DGPRF_RNG_HYPER, chain, slot);
    const float mn = beta * m - (h * N) * g + sqrtf(2.0f * (1.0f - beta) * T * M) * eps;
    *m_out = mn;
    return v + (h * (1.0f / M)) * mn;
  };
  if (hb == k.n_blocks - 1) {  // Gaussian lik_log_var (likelihoods/gaussian.py:12)
    const bool lik_tr = (k.flags & DGPRF_HYP_LIK) && k.likelihood == DGPRF_LIK_GAUSSIAN;
    if (GONLY) {  // slots no workgroup owns (padding, groups that do not train) read as 0
      for (int64_t s = tid; s < k.hyp_total; s += NT) {
        bool owned = s < L ? (k.flags & DGPRF_HYP_KERNEL) != 0 : (s == L && lik_tr);
        for (int q = 0; q < L; ++q) {
          owned |= (k.flags & DGPRF_HYP_KERNEL) && s >= k.lis_off[q] && s < k.lis_off[q] + k.d[q];
          owned |= (k.flags & DGPRF_HYP_MEAN) && s >= k.mean_off[q] && s < k.mean_off[q] + k.d[q];
        }
        if (!owned) gout[s] = 0.f;
      }
    }
    if (lik_tr && tid == 0) {
      const float* hpl = k.ws + (int64_t)chain * a.ws_cs + k.hpl_off;
      float s = 0.f;
      for (int rt = 0; rt < a.n_rt; ++rt) s += hpl[rt];
      const float v0 = hyp[L];
      float mn = 0.f;
      const float v = upd(L, s + v0 / N, v0, GONLY ? 0.f : hm[L], 24, &mn);
      if (!GONLY) {
        hm[L] = mn;
        hyp[L] = v;
        k.der[(int64_t)chain * k.der_cs + DGPRF_MAX_LAYERS] = expf(v);
      }
    }
    return;
  }
  int l = 0;
  for (int q = 1; q < L; ++q)
    if (hb >= k.b0[q]) l = q;
  const int j = hb - k.b0[l], d = k.d[l], R = k.R[l], nv = 2 * d + 1, hs = (nv + 3) & ~3;
  const int Q = hs >> 2, ns = k.ns[l], P = a.n_rt * ns, RG = Q >= NT ? 1 : NT / Q;
  const bool kern = (k.flags & DGPRF_HYP_KERNEL) != 0, mean = (k.flags & DGPRF_HYP_MEAN) != 0;
  const int64_t lis = k.lis_off[l], mo = k.mean_off[l];
  // LDS: totals | old values | old momenta | new values | exp(new lis) | row-group partials | tree
  float* tot = sm;
  float* ov = tot + hs;   // [0] log_amp, [1+k] log_inv_ls, [1+d+k] mean
  float* om = ov + hs;
  float* nvv = om + hs;
  float* els = nvv + hs;  // exp(new lis)[d]
  float* part = els + hs;                       // [RG][hs]
  float* red = part + (4 * NT > hs ? 4 * NT : hs);  // [NT] tree, [NT] last-arrival flag
  auto slot_of = [&](int e) -> int64_t { return e == 0 ? (int64_t)l : (e <= d ? lis + e - 1 : mo + e - 1 - d); };
  // (0) z of this workgroup's Omega slice and the old values / momenta first: independent loads
  float* omg = k.omega + (int64_t)chain * k.om_cs + k.om_off[l];
  const int64_t n_el = (int64_t)d * R, base = (int64_t)j * HYP_EPB;
  f4 zv[4];
  if (!GONLY) {
    const rsrc_t rz = make_rsrc(k.z + k.om_off[l], n_el);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t i = base + 4 * (tid + NT * u);
      zv[u] = bload4(rz, i < n_el ? (uint32_t)(i * 4) : DGPRF_OOB);
    }
  }
  for (int e = tid; e < 1 + 2 * d; e += NT) {
    const int64_t s = slot_of(e);
    ov[e] = hyp[s];
    om[e] = GONLY ? 0.f : hm[s];
  }
  __syncthreads();  // every old value of this workgroup has been read
  DGPRF_STAMP(sb, 1);
  // arrival on the layer's counter (its return overlaps the partial loads below)
  unsigned* cnt = reinterpret_cast<unsigned*>(const_cast<float*>(k.ws) + (int64_t)chain * a.ws_cs +
                                              k.cnt_off) + l;
  unsigned arrived = 0u;
  if (!GONLY && k.nb[l] > 1 && tid == 0) arrived = atomicAdd(cnt, 1u);
  // (1) partial row sums: up to HYP_U loads per lane in flight, summed in row order
  // rows p = rt * ns + sl of a row group advance by RG: (rt, sl) tracked without divisions
  constexpr int HYP_U = 8;
  const float* hp = k.ws + (int64_t)chain * a.ws_cs + k.hpp_off[l];
  const rsrc_t rh = make_rsrc(hp, (int64_t)a.n_rt * NSM * hs);
  const int st_rt = RG / ns, st_sl = RG - st_rt * ns;
  for (int i = tid; i < RG * Q; i += NT) {
    const int q = i % Q, rg = i / Q;
    int rt = rg / ns, sl = rg - rt * ns;
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int p0 = rg; p0 < P; p0 += HYP_U * RG) {
      f4 v[HYP_U];
#pragma unroll
      for (int u = 0; u < HYP_U; ++u) {
        v[u] = bload4(rh, rt < a.n_rt ? (uint32_t)(((rt * NSM + sl) * hs + 4 * q) * 4) : DGPRF_OOB);
        rt += st_rt;
        sl += st_sl;
        if (sl >= ns) {
          sl -= ns;
          ++rt;
        }
      }
#pragma unroll
      for (int u = 0; u < HYP_U; ++u) acc += v[u];
    }
    *reinterpret_cast<f4*>(part + rg * hs + 4 * q) = acc;
  }
  DGPRF_STAMP(sb, 2);
  __syncthreads();
  for (int e = tid; e < nv; e += NT) {
    float s = 0.f;
    for (int rg = 0; rg < RG; ++rg) s += part[rg * hs + e];
    tot[e] = s;
  }
  __syncthreads();
  DGPRF_STAMP(sb, 3);
  // (2) new values: one update site for every slot (scalar lis: one slot, broadcast after)
  const bool scalar_lis = kern && !k.ard[l];
  float gsc = 0.f;
  if (scalar_lis) {  // one length scale: its gradient sums over the d dims (fixed-order tree)
    float sp = 0.f;
    for (int kk = tid; kk < d; kk += NT) sp += expf(ov[1 + kk]) * tot[kk];
    red[tid] = sp;
    __syncthreads();
    for (int w = NT / 2; w > 0; w >>= 1) {
      if (tid < w) red[tid] += red[tid + w];
      __syncthreads();
    }
    gsc = red[0];
  }
  for (int e = tid; e < 1 + 2 * d; e += NT) {
    float v = ov[e], mn = om[e];
    bool tr;
    float g;
    int midx;
    int64_t slot;
    if (e == 0) {
      tr = kern;
      g = tot[2 * d];
      midx = l;
      slot = l;
    } else if (e <= d) {
      tr = kern && (!scalar_lis || e == 1);
      g = scalar_lis ? gsc : expf(ov[e]) * tot[e - 1];
      midx = 8 + l;
      slot = lis + e - 1;
    } else {
      tr = mean;
      g = tot[e - 1];
      midx = 16 + l;
      slot = mo + e - 1 - d;
    }
    if (tr) v = upd(slot, g + ov[e] / N, ov[e], om[e], midx, &mn);
    nvv[e] = v;
    om[e] = mn;
  }
  if (scalar_lis) {
    __syncthreads();
    for (int kk = 1 + tid; kk < d; kk += NT) {
      nvv[1 + kk] = nvv[1];
      om[1 + kk] = om[1];
      if (GONLY) gout[lis + kk] = gsc + ov[1] / N;
    }
  }
  if (GONLY) return;
  __syncthreads();
  DGPRF_STAMP(sb, 4);
  for (int kk = tid; kk < d; kk += NT) els[kk] = expf(nvv[1 + kk]);
  // (3) the last workgroup of the layer to arrive stores the new hyp / hmom
  bool last = k.nb[l] == 1;
  if (!last) {
    if (tid == 0) {
      const bool lst = arrived == (unsigned)k.nb[l] - 1u;
      if (lst) *cnt = 0u;
      red[NT] = lst ? 1.f : 0.f;
    }
    __syncthreads();
    last = red[NT] != 0.f;
  } else {
    __syncthreads();
  }
  if (last) {
    for (int e = tid; e < 1 + 2 * d; e += NT) {
      const bool tr = e == 0 ? kern : (e <= d ? kern : mean);
      if (!tr) continue;
      const int64_t s = slot_of(e);
      hyp[s] = nvv[e];
      hm[s] = om[e];
    }
  }
  DGPRF_STAMP(sb, 5);
  // (4) this workgroup's slice of Omega_l and c_l (layers/rf_layers.py:44,90)
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int64_t i = base + 4 * (tid + NT * u);
    if (i >= n_el) continue;
    f4 o;
    int kk = (int)((uint32_t)i / (uint32_t)R), rc = (int)i - kk * R;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int kc = kk < d ? kk : d - 1;
      o[c] = els[kc] * zv[u][c] + nvv[1 + d + kc];
      for (++rc; rc >= R; rc -= R) ++kk;
    }
    if (i + 3 < n_el) {
      *reinterpret_cast<f4*>(omg + i) = o;
    } else {
      for (int c = 0; c < 4 && i + c < n_el; ++c) omg[i + c] = o[c];
    }
  }
  if (j == 0 && tid == 0) {
    const float amp = expf(nvv[0]), sq = sqrtf((float)R);
    k.der[(int64_t)chain * k.der_cs + l] = k.kind[l] == DGPRF_RBF ? amp / sq : (sqrtf(2.f) * amp) / sq;
  }
#ifdef DGPRF_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  DGPRF_STAMP(sb, 14);
}

template <bool GIN, bool GONLY, bool XI, bool CYC>
__global__ __launch_bounds__(UPD_THREADS) void k_step_update(const UpdK a) {
  extern __shared__ __attribute__((aligned(16))) float usm[];
  const int chain = blockIdx.y;
  const int stamp_base = 16 * 4096 + blockIdx.y * gridDim.x + blockIdx.x;
  DGPRF_STAMP(stamp_base, 0);
  if (!GIN && (int)blockIdx.x < a.hyp_blocks) {  // full_bayesian=True hyper-parameters
    hyper_block<GONLY, XI, CYC>(a, (int)blockIdx.x, chain, usm, stamp_base);
    return;
  }
  const int bx = (int)blockIdx.x - a.hyp_blocks;
  if (bx >= a.upd_blocks) {  // dedicated blocks: rows of step t+1 (off the path)
    const int64_t t = *a.step + (int64_t)a.step_offset;
    if (a.d_in > GATHER_WIDE) {  // one-wave blocks: one row each
      const int b = bx - a.upd_blocks;
      if (a.gather_next && b < a.B)
        gather_row_wave(a.bd, a.B, a.d_in, a.yb_cols, a.xb + (int64_t)chain * a.ws_cs,
                        a.yb + (int64_t)chain * a.ws_cs, chain, t + 1, b, threadIdx.x);
      return;
    }
    const int b = (bx - a.upd_blocks) * UPD_THREADS + threadIdx.x;
    if (a.gather_next && b < a.B)
      gather_row(a.bd, a.B, a.d_in, a.yb_cols, a.xb + (int64_t)chain * a.ws_cs,
                 a.yb + (int64_t)chain * a.ws_cs, chain, t + 1, b);
    return;
  }
  // four packed parameters per lane (one counter quad of Philox normals, 16-byte loads); layer
  // offsets are multiples of 4, so a quad never straddles two layers
  const int e0 = 4 * (bx * UPD_THREADS + (int)threadIdx.x);
  const uint32_t off = (uint32_t)e0 * 4u;
  const int64_t cw = (int64_t)chain * a.w_total;
  const rsrc_t rth = make_rsrc(a.theta + cw, a.w_total);
  const f4 th = bload4(rth, off);
  f4 m = f4zero(), gr;
  if (!GONLY) m = bload4(make_rsrc(a.mom + cw, a.w_total), off);
  if (GIN) {
    gr = bload4(make_rsrc(a.grad_in + cw, a.w_total), off);
  } else {
    // sum the row-tile gW partials in a fixed order: groups of 16 independent loads
    const rsrc_t rs = make_rsrc(a.gwp + (int64_t)chain * a.ws_cs, (int64_t)a.n_rt * a.w_total);
    f4 sacc = f4zero();
    for (int rt0 = 0; rt0 < a.n_rt_pad; rt0 += 16) {
      f4 v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = bload4(rs, (uint32_t)(((rt0 + j) * a.w_total + e0) * 4));
#pragma unroll
      for (int j = 0; j < 16; ++j) sacc += v[j];
    }
    gr = sacc;
  }
  int layer = 0;
#pragma unroll
  for (int l = 1; l < DGPRF_MAX_LAYERS; ++l)
    if (l < a.n_layers && e0 >= a.lo[l]) layer = l;
  // layer padding between align4 offsets stays untouched: live elements of the quad
  const int nlive = min(max(a.hi[layer] - e0, 0), 4);
  auto store = [&](float* p, f4 v) {
    if (nlive == 4) {
      st4(p, v);
    } else {
      for (int k = 0; k < nlive; ++k) p[k] = v[k];
    }
  };
  const UpdateDev& ud = a.ud;
  const float N = ud.data_size;
  // dU/dW = W/N (prior N(0,1), models/dgp.py:129-136,171) + Phi^T dF (likelihood)
  if (!GIN) gr = th / N + gr;
  if (GONLY) {
    store(a.grad_out + (int64_t)chain * a.grad_cs + e0, gr);
    return;
  }
  const float M = a.mass[chain * a.n_layers + layer];
  // the step counter (written by the previous step's k_advance) is read only now, after the
  // parameter and partial loads are in flight
  const int64_t t = *a.step + (int64_t)a.step_offset;
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
  store(a.mom + cw + e0, mn);
  store(a.theta + cw + e0, th + (h * (1.0f / M)) * mn);
#ifdef DGPRF_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  DGPRF_STAMP(stamp_base, 14);
}


// random_fixed=False (layers/rf_layers.py:39-41): Omega_l = exp(lis_l)[:,None] z + mean_l[:,None]
// with z ~ N(0,1) drawn for this step — Philox (seed, sub = step, DGPRF_RNG_Z, tag = 1 + l + 16
// chain), element i of the layer at counter quad i / 4 — for the fresh layers.  One thread per
// 4 elements; chain blockIdx.y writes its own workspace copy.
__global__ void k_fresh_omega(const dgprf_plan_t pl, const float* __restrict__ hyp, float* ws,
                              const int64_t* step, uint64_t seed, int32_t step_offset) {
  const int chain = blockIdx.y;
  const int64_t i0 = 4 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  if (i0 >= pl.omega_total) return;
  int layer = 0;
  for (int l = 1; l < pl.n_layers; ++l)
    if (i0 >= pl.omega_off[l]) layer = l;
  if (!((pl.fresh_z >> layer) & 1)) return;
  const float* h = hyp + (pl.hyp_per_chain ? (int64_t)chain * pl.hyp_total : 0);
  float* om = ws + (int64_t)chain * pl.ws_chain + pl.omf_off;
  const int64_t n_l = (int64_t)pl.d[layer] * pl.n_rf[layer];
  const int64_t j0 = i0 - pl.omega_off[layer];  // omega_off is a multiple of 4
  const int64_t t = *step + step_offset;
  const f4 z = philox_normal4(seed, (uint64_t)t, DGPRF_RNG_Z, 1u + layer + 16u * chain,
                              (uint32_t)(j0 >> 2));
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int64_t j = j0 + c;
    if (j < n_l) {
      const int k = (int)(j / pl.n_rf[layer]);
      om[pl.omega_off[layer] + j] = expf(h[pl.lis_off[layer] + k]) * z[c] + h[pl.mean_off[layer] + k];
    }
  }
}

__global__ void k_advance(int64_t* step, int64_t by) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *step += by;
}

// ------------------------------------------------------------------------- host helpers
// ------------------------------------------------------------------------- wide first layer
// A_1 = X Omega_1 for a first layer with d > 32 (BASELINE config 4: d = 784, R = 4096), written
// to the workspace for the layer-0 forward and backward, which would otherwise each run a d-long
// dependent k-step loop per 16-feature chunk.  One workgroup = 32 rows x 64 features; its 4 waves
// own 16 x 32 sub-tiles (2 accumulators); K runs in LDS-staged blocks of 32 (X block [32][33],
// Omega block [32][68]), the next block's loads in flight while the current one computes.  Rows
// >= B and k >= d are staged as zeros.
struct AgemmK {
  const float* xrows;  // [B][d_in] of chain 0 (stride xrow_cs)
  const float* om;     // Omega_1 [d][R] of chain 0 (stride om_cs)
  float* aout;         // [align32(B)][R] of chain 0 (stride ws_cs)
  int64_t xrow_cs, om_cs, ws_cs;
  int32_t B, d, R, d_in;
};
constexpr int AG_KB = 32, AG_XST = 33, AG_OST = 68;

__global__ __launch_bounds__(256) void k_step_agemm(const AgemmK a) {
  __shared__ float xsm[2][32 * AG_XST];
  __shared__ __attribute__((aligned(16))) float osm[2][AG_KB * AG_OST];
  const int chain = blockIdx.z;
  const int rb = blockIdx.y * 32, fb = blockIdx.x * 64;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 15, lq = lane >> 4;
  const int wr = wave >> 1, wc = wave & 1;
  const float* X = a.xrows + (int64_t)chain * a.xrow_cs;
  const float* om = a.om + (int64_t)chain * a.om_cs;
  const int d = a.d, R = a.R;
  // staging assignment: X block: 4 scalars per thread (row tid >> 3, k (tid & 7) * 4 + q);
  // Omega block: 2 float4 per thread (k = e >> 4, features 4 (e & 15))
  const int xr = tid >> 3, xk = (tid & 7) * 4;
  const rsrc_t rx = make_rsrc(X, (int64_t)a.B * a.d_in);
  const rsrc_t ro = make_rsrc(om, (int64_t)d * R);
  float xv[4];
  f4 ov[2];
  auto load = [&](int kb) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = rb + xr, k = kb + xk + q;
      xv[q] = bload1(rx, row < a.B && k < d ? (uint32_t)(((int64_t)row * a.d_in + k) * 4) : DGPRF_OOB);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int e = tid + 256 * j, k = kb + (e >> 4), f = fb + 4 * (e & 15);
      ov[j] = bload4(ro, k < d && f < R ? (uint32_t)(((int64_t)k * R + f) * 4) : DGPRF_OOB);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 4; ++q) xsm[buf][xr * AG_XST + xk + q] = xv[q];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int e = tid + 256 * j;
      *reinterpret_cast<f4*>(&osm[buf][(e >> 4) * AG_OST + 4 * (e & 15)]) = ov[j];
    }
  };
  f4 acc0 = f4zero(), acc1 = f4zero();
  const int nkb = (d + AG_KB - 1) / AG_KB;
  load(0);
  store(0);
  __syncthreads();
  for (int kb = 0; kb < nkb; ++kb) {
    const int buf = kb & 1;
    if (kb + 1 < nkb) load((kb + 1) * AG_KB);
    const float* xb = &xsm[buf][(wr * 16 + lr) * AG_XST + lq];
    const float* ob = &osm[buf][lq * AG_OST + wc * 32 + lr];
#pragma unroll
    for (int ks = 0; ks < AG_KB / 4; ++ks) {
      const float xa = xb[4 * ks];
      acc0 = mfma16(xa, ob[4 * ks * AG_OST], acc0);
      acc1 = mfma16(xa, ob[4 * ks * AG_OST + 16], acc1);
    }
    if (kb + 1 < nkb) store(buf ^ 1);
    __syncthreads();
  }
  // acc[r] = A[row wr*16 + 4lq + r][feature wc*32 + n*16 + lr]
  float* out = a.aout + (int64_t)chain * a.ws_cs;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t row = rb + wr * 16 + 4 * lq + r;
    const int f = fb + wc * 32 + lr;
    if (f < R) out[row * R + f] = acc0[r];
    if (f + 16 < R) out[row * R + f + 16] = acc1[r];
  }
}

LayerK make_layer_k(const dgprf_plan_t& pl, const StepDev& sd, int l, int& lds_floats,
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
  a.xrows = direct ? sd.bd.X : sd.ws + (sd.xb_sel ? pl.xb_alt_off : pl.xb_off);
  a.yrows = direct ? sd.bd.Y : sd.ws + (sd.xb_sel ? pl.yb_alt_off : pl.yb_off);
  a.xrow_cs = direct ? 0 : pl.ws_chain;
  a.yrow_cs = direct ? 0 : pl.ws_chain;
  a.y_cols = direct ? sd.bd.y_cols : pl.yb_cols;
  a.cptr = sd.der + l;
  a.varptr = sd.der + DGPRF_MAX_LAYERS;
  a.om_cs = fresh ? pl.ws_chain : sd.om_cs;
  a.der_cs = sd.der_cs;
  a.w_cs = pl.w_total;
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
  step_lds(a.d, a.g, a, lds_floats, nwb);
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
  a.n_rt = pl.n_row_tiles;
  a.ns = pl.ns[l];
  a.rt_per_xcd = (pl.n_row_tiles + 7) / 8;
  // full_bayesian=True: z rows, hyper partials, per-wave LDS sums [4][round4(2d+1)]
  a.a0 = (l == 0 && pl.a0_off >= 0 && sd.ws) ? sd.ws + pl.a0_off : nullptr;
  a.z = sd.z ? sd.z + pl.omega_off[l] : nullptr;
  a.hp = sd.ws + pl.hpp_off[l];
  a.hpl = sd.ws + pl.hpl_off;
  a.lik_fb = (pl.hyp_flags & DGPRF_HYP_LIK) != 0 && pl.likelihood == DGPRF_LIK_GAUSSIAN;
  // whole-slice staging for the backward (used only where dPhi / dX need W and Omega)
  a.kind_rbf = pl.kind[l] == DGPRF_RBF;
  a.pad_w = 0;
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
  // fused update: off unless the launcher sets it up (fill_fused)
  a.main_blocks = 8 * a.rt_per_xcd * a.ns;
  a.smap = a.pad_s = 0;
  a.pend = a.upd_blocks = a.gat_blocks = 0;
  a.th0 = a.mo0 = nullptr;
  a.mass = nullptr;
  a.step = sd.step;
  a.gwb = nullptr;
  a.tick = nullptr;
  a.seed = sd.seed;
  a.n_layers = pl.n_layers;
  a.pend_lo = a.upd_layer = a.upd_lo = a.upd_hi = a.upd_t_off = a.gat_t_off = 0;
  std::memset(&a.ud, 0, sizeof(a.ud));
  std::memset(&a.bd, 0, sizeof(a.bd));
  a.xb_next = a.yb_next = nullptr;
  a.yb_cols = pl.yb_cols;
  a.pad_f = 0;
  return a;
}

// The state the fused-update paths of a layer launch read (plan.fused_update).
void fill_fused(LayerK& a, const dgprf_plan_t& pl, const StepDev& sd, const UpdateDev& ud) {
  a.th0 = sd.theta;
  a.mo0 = sd.mom;
  a.mass = sd.mass;
  a.gwb = sd.ws + pl.gwp_off;
  a.tick = reinterpret_cast<unsigned*>(sd.ws + pl.tick_off);
  a.ud = ud;
}

// Layer `layer`'s packed W range for the update workgroups of `threads` threads.
void set_update_range(LayerK& a, const dgprf_plan_t& pl, int layer, int t_off, int threads = 256) {
  a.upd_layer = layer;
  a.upd_lo = (int32_t)pl.w_off[layer];
  a.upd_hi = (int32_t)(pl.w_off[layer] + (int64_t)pl.P[layer] * pl.n_gp[layer]);
  a.upd_blocks = (a.upd_hi - a.upd_lo + 4 * threads - 1) / (4 * threads);
  a.upd_t_off = t_off;
}

#define DGPRF_KS_NOT_DISPATCH(KERNEL)                                                              \
  template <int KS, int NOT, bool G1>                                                              \
  void KERNEL##_launch3(bool rbf, dim3 grid, size_t lds, hipStream_t s, const LayerK& a) {         \
    if (rbf) {                                                                                     \
      dgprf::set_lds_limit((const void*)KERNEL<KS, NOT, true, G1>, lds);                           \
      hipLaunchKernelGGL((KERNEL<KS, NOT, true, G1>), grid, dim3(256), lds, s, a);                 \
    } else {                                                                                       \
      dgprf::set_lds_limit((const void*)KERNEL<KS, NOT, false, G1>, lds);                          \
      hipLaunchKernelGGL((KERNEL<KS, NOT, false, G1>), grid, dim3(256), lds, s, a);                \
    }                                                                                              \
  }                                                                                                \
  template <int KS>                                                                                \
  void KERNEL##_launch2(int g, bool rbf, dim3 grid, size_t lds, hipStream_t s,                     \
                        const LayerK& a) {                                                         \
    const int NOT = (g + 15) >> 4;                                                                 \
    if (g == 1) KERNEL##_launch3<KS, 1, true>(rbf, grid, lds, s, a);                               \
    else switch (NOT) {                                                                            \
      case 1: KERNEL##_launch3<KS, 1, false>(rbf, grid, lds, s, a); break;                         \
      case 2: KERNEL##_launch3<KS, 2, false>(rbf, grid, lds, s, a); break;                         \
      case 3: KERNEL##_launch3<KS, 3, false>(rbf, grid, lds, s, a); break;                         \
      default: KERNEL##_launch3<KS, 4, false>(rbf, grid, lds, s, a); break;                        \
    }                                                                                              \
  }                                                                                                \
  void KERNEL##_launch(int d, int g, bool rbf, dim3 grid, size_t lds, hipStream_t s,               \
                       const LayerK& a) {                                                          \
    if (d <= 4) KERNEL##_launch2<1>(g, rbf, grid, lds, s, a);                                      \
    else if (d <= 8) KERNEL##_launch2<2>(g, rbf, grid, lds, s, a);                                 \
    else if (d <= 16) KERNEL##_launch2<4>(g, rbf, grid, lds, s, a);                                \
    else if (d <= 32) KERNEL##_launch2<8>(g, rbf, grid, lds, s, a);                                \
    else KERNEL##_launch2<0>(g, rbf, grid, lds, s, a);                                             \
  }

// forward: KS x NOT x RBF x G1 (x PEND for the narrow layers the fused update covers: NOT == 1) x
// waves per workgroup (8 / 16 for slices of >= 2 chunks per wave: two / four waves per SIMD hide
// each other's MFMA / load latency; 4 otherwise and with PEND)
template <int KS, int NOT, bool G1>
void k_step_fwd_launch3(bool rbf, bool pend, int nw, dim3 grid, size_t lds, hipStream_t s,
                        const LayerK& a) {
#define DGPRF_FWD(R_, P_, W_)                                                                  \
  do {                                                                                        \
    dgprf::set_lds_limit((const void*)k_step_fwd<KS, NOT, R_, G1, P_, W_>, lds);             \
    hipLaunchKernelGGL((k_step_fwd<KS, NOT, R_, G1, P_, W_>), grid, dim3(64 * W_), lds, s, a); \
  } while (0)
  if (pend && NOT == 1) {
    if (rbf) DGPRF_FWD(true, NOT == 1, 4);
    else DGPRF_FWD(false, NOT == 1, 4);
  } else if (nw == 16) {
    if (rbf) DGPRF_FWD(true, false, 16);
    else DGPRF_FWD(false, false, 16);
  } else if (nw == 8) {
    if (rbf) DGPRF_FWD(true, false, 8);
    else DGPRF_FWD(false, false, 8);
  } else {
    if (rbf) DGPRF_FWD(true, false, 4);
    else DGPRF_FWD(false, false, 4);
  }
#undef DGPRF_FWD
}
template <int KS>
void k_step_fwd_launch2(int g, bool rbf, bool pend, int nw, dim3 grid, size_t lds, hipStream_t s,
                        const LayerK& a) {
  const int NOT = (g + 15) >> 4;
  if (g == 1) k_step_fwd_launch3<KS, 1, true>(rbf, pend, nw, grid, lds, s, a);
  else if (NOT == 1) k_step_fwd_launch3<KS, 1, false>(rbf, pend, nw, grid, lds, s, a);
  else if (NOT == 2) k_step_fwd_launch3<KS, 2, false>(rbf, false, nw, grid, lds, s, a);
  else if (NOT == 3) k_step_fwd_launch3<KS, 3, false>(rbf, false, nw, grid, lds, s, a);
  else k_step_fwd_launch3<KS, 4, false>(rbf, false, nw, grid, lds, s, a);
}
void k_step_fwd_launch(int d, int g, bool rbf, bool pend, int nw, dim3 grid, size_t lds,
                       hipStream_t s, const LayerK& a) {
  if (d <= 4) k_step_fwd_launch2<1>(g, rbf, pend, nw, grid, lds, s, a);
  else if (d <= 8) k_step_fwd_launch2<2>(g, rbf, pend, nw, grid, lds, s, a);
  else if (d <= 16) k_step_fwd_launch2<4>(g, rbf, pend, nw, grid, lds, s, a);
  else if (d <= 32) k_step_fwd_launch2<8>(g, rbf, pend, nw, grid, lds, s, a);
  else k_step_fwd_launch2<0>(g, rbf, false, nw, grid, lds, s, a);
}

// backward: KS x NOT x RBF x G1 x FB x waves per workgroup (8: W-only with whole-slice staging)
// x FUSED (W-only, 4 waves)
template <int KS, int NOT, bool G1>
void k_step_bwd_launch3(bool rbf, bool fb, bool w8, bool fu, dim3 grid, size_t lds, hipStream_t s,
                        const LayerK& a) {
#define DGPRF_BWD(R_, F_, W_, U_)                                                                 \
  do {                                                                                           \
    dgprf::set_lds_limit((const void*)k_step_bwd<KS, NOT, R_, G1, F_, W_, U_>, lds);            \
    hipLaunchKernelGGL((k_step_bwd<KS, NOT, R_, G1, F_, W_, U_>), grid, dim3(64 * W_), lds, s, a); \
  } while (0)
  if (rbf) {
    if (fb) DGPRF_BWD(true, true, 4, false);
    else if (fu) DGPRF_BWD(true, false, 4, true);
    else if (w8) DGPRF_BWD(true, false, 8, false);
    else DGPRF_BWD(true, false, 4, false);
  } else {
    if (fb) DGPRF_BWD(false, true, 4, false);
    else if (fu) DGPRF_BWD(false, false, 4, true);
    else if (w8) DGPRF_BWD(false, false, 8, false);
    else DGPRF_BWD(false, false, 4, false);
  }
#undef DGPRF_BWD
}
template <int KS>
void k_step_bwd_launch2(int g, bool rbf, bool fb, bool w8, bool fu, dim3 grid, size_t lds,
                        hipStream_t s, const LayerK& a) {
  const int NOT = (g + 15) >> 4;
  if (g == 1) k_step_bwd_launch3<KS, 1, true>(rbf, fb, w8, fu, grid, lds, s, a);
  else if (NOT == 1) k_step_bwd_launch3<KS, 1, false>(rbf, fb, w8, fu, grid, lds, s, a);
  else if (NOT == 2) k_step_bwd_launch3<KS, 2, false>(rbf, fb, w8, fu, grid, lds, s, a);
  else if (NOT == 3) k_step_bwd_launch3<KS, 3, false>(rbf, fb, w8, fu, grid, lds, s, a);
  else k_step_bwd_launch3<KS, 4, false>(rbf, fb, w8, fu, grid, lds, s, a);
}
void k_step_bwd_launch(int d, int g, bool rbf, bool fb, bool w8, bool fu, dim3 grid, size_t lds,
                       hipStream_t s, const LayerK& a) {
  if (d <= 4) k_step_bwd_launch2<1>(g, rbf, fb, w8, fu, grid, lds, s, a);
  else if (d <= 8) k_step_bwd_launch2<2>(g, rbf, fb, w8, fu, grid, lds, s, a);
  else if (d <= 16) k_step_bwd_launch2<4>(g, rbf, fb, w8, fu, grid, lds, s, a);
  else if (d <= 32) k_step_bwd_launch2<8>(g, rbf, fb, w8, fu, grid, lds, s, a);
  else k_step_bwd_launch2<0>(g, rbf, fb, w8, fu, grid, lds, s, a);
}

}  // namespace

#ifdef DGPRF_STAMPS
__device__ unsigned long long g_dgprf_stamps[17 * 4096 * DGPRF_STAMP_SLOTS];
extern "C" int dgprf_debug_read_stamps(unsigned long long* host, long long n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_dgprf_stamps), (size_t)n * 8, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : -3;
}
extern "C" int dgprf_debug_clear_stamps(void) {
  static unsigned long long zeros[17 * 4096 * DGPRF_STAMP_SLOTS];
  return hipMemcpyToSymbol(HIP_SYMBOL(g_dgprf_stamps), zeros, sizeof(zeros), 0,
                           hipMemcpyHostToDevice) == hipSuccess ? 0 : -3;
}
#endif

namespace dgprf {

// A_1 = X Omega_1 of the step's gathered rows into the workspace (plan.a0_off): hipBLASLt, or
// k_step_agemm when the library has no candidate for the shape (or its handle would have to be
// created under stream capture).
hipError_t launch_step_agemm(const dgprf_plan_t& pl, const StepDev& sd, hipStream_t s) {
  int lds_floats = 0;
  const LayerK a = make_layer_k(pl, sd, 0, lds_floats);
  if (!a.a0) return hipSuccess;
  if (blas_agemm(a.xrows, pl.batch, pl.d_in, pl.d[0], a.om, pl.n_rf[0], sd.ws + pl.a0_off,
                 pl.n_chains, a.xrow_cs, a.om_cs, pl.ws_chain, s))
    return hipSuccess;
  AgemmK g;
  g.xrows = a.xrows;
  g.om = a.om;
  g.aout = sd.ws + pl.a0_off;
  g.xrow_cs = a.xrow_cs;
  g.om_cs = a.om_cs;
  g.ws_cs = pl.ws_chain;
  g.B = pl.batch;
  g.d = pl.d[0];
  g.R = pl.n_rf[0];
  g.d_in = pl.d_in;
  dim3 ggrid((unsigned)((g.R + 63) / 64), (unsigned)((g.B + 31) / 32), pl.n_chains);
  hipLaunchKernelGGL(k_step_agemm, ggrid, dim3(256), 0, s, g);
  return hipGetLastError();
}

hipError_t launch_step_fwd(const dgprf_plan_t& pl, const StepDev& sd, int layer, hipStream_t s,
                           const UpdateDev* ud, bool pend) {
  pend = pend && ud && layer == 0 && pl.fused_update == 1 && pl.n_gp[0] <= 16 && pl.d[0] <= 32;
  // 8 waves per workgroup when every wave still gets >= 2 chunks and no pending update is applied
  // (config 3, cpw = 2: one chunk per wave measured slower, 37.6 vs 35.9 us/step)
  const bool w8 = !pend && pl.cpw[layer] >= 4 && pl.cpw[layer] % 2 == 0;
  // 16 waves (four per SIMD) when every wave still gets >= 2 chunks (config 5, cpw = 8:
  // 104.4 -> 102.4 us/step; with one chunk per wave, config 4, no gain)
  const int nwf = (w8 && pl.cpw[layer] % 8 == 0) ? 16 : (w8 ? 8 : 4);
  int lds_floats = 0;
  LayerK a = make_layer_k(pl, sd, layer, lds_floats, false, nwf);
  if (pend) {  // the previous step's W_1 update, applied by this forward (its step offset - 1)
    fill_fused(a, pl, sd, *ud);
    a.pend = 1;
    a.pend_lo = (int32_t)pl.w_off[0];
    a.upd_t_off = sd.step_offset - 1;
    lds_floats = max(lds_floats, a.stg_off + 4096 + 4);  // the new slice + the last-arrival flag
    a.smap = 1;
    a.main_blocks = 8 * ((a.ns + 7) / 8) * a.n_rt;
  }
  if (a.a0) {  // wide first layer: A_1 = X Omega_1 first
    const hipError_t e = launch_step_agemm(pl, sd, s);
    if (e != hipSuccess) return e;
  }
  dim3 grid(a.main_blocks, 1, pl.n_chains);
  k_step_fwd_launch(pl.d[layer], pl.n_gp[layer], pl.kind[layer] == DGPRF_RBF, pend, nwf, grid,
                    (size_t)lds_floats * sizeof(float), s, a);
  return hipGetLastError();
}

hipError_t launch_step_bwd(const dgprf_plan_t& pl, const StepDev& sd, int layer, hipStream_t s,
                           const UpdateDev* ud, bool gather_next) {
  // 8 waves per workgroup for W-only steps whose slices are staged whole (a.wstage); not with the
  // fused update's extra workgroups (measured slower)
  const bool fused = ud && pl.fused_update;
  bool w8 = !sd.full_bayes && !fused && pl.cpw[layer] % 4 == 0;
  int lds_floats = 0;
  LayerK a = make_layer_k(pl, sd, layer, lds_floats, /*bwd=*/true, w8 ? 8 : 4);
  if (w8 && !a.wstage) {  // the slice image does not fit next to 8 waves' rows: 4 waves
    w8 = false;
    lds_floats = 0;
    a = make_layer_k(pl, sd, layer, lds_floats, /*bwd=*/true, 4);
  }
  if (fused) {
    fill_fused(a, pl, sd, *ud);
    // extra workgroups: W_{l+2}'s update from the gW partials layer l+1's backward just wrote
    const int nt = 256;
    if (layer + 1 < pl.n_layers) set_update_range(a, pl, layer + 1, sd.step_offset, nt);
    // and, in the last layer's backward, step t+1's rows into the other buffer
    if (gather_next && layer == pl.n_layers - 1 && sd.bd.mode == DGPRF_BATCH_EPOCH) {
      a.gat_blocks = pl.d_in > GATHER_WIDE ? (pl.batch + nt / 64 - 1) / (nt / 64)
                                           : (pl.batch + nt - 1) / nt;
      a.bd = sd.bd;
      a.xb_next = sd.ws + (sd.xb_sel ? pl.xb_off : pl.xb_alt_off);
      a.yb_next = sd.ws + (sd.xb_sel ? pl.yb_off : pl.yb_alt_off);
      a.gat_t_off = sd.step_offset + 1;
    }
  }
  dim3 grid(a.main_blocks + a.upd_blocks + a.gat_blocks, 1, pl.n_chains);
  k_step_bwd_launch(pl.d[layer], pl.n_gp[layer], pl.kind[layer] == DGPRF_RBF, sd.full_bayes != 0,
                    w8, fused, grid, (size_t)lds_floats * sizeof(float), s, a);
  return hipGetLastError();
}

hipError_t launch_layer_update(const dgprf_plan_t& pl, const StepDev& sd, const UpdateDev& ud,
                               int layer, hipStream_t s) {
  int lds_floats = 0;
  LayerK a = make_layer_k(pl, sd, layer, lds_floats);
  fill_fused(a, pl, sd, ud);
  set_update_range(a, pl, layer, sd.step_offset);
  hipLaunchKernelGGL(k_layer_update, dim3(a.upd_blocks, 1, pl.n_chains), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_step_update(const dgprf_plan_t& pl, const StepDev& sd, const UpdateDev& ud,
                              const float* grad_in, hipStream_t s, bool gather_next) {
  if (pl.w_total >= (int64_t)1 << 30 || (int64_t)pl.n_rt_pad * pl.w_total >= (int64_t)1 << 29)
    return hipErrorInvalidValue;  // 32-bit buffer offsets
  UpdK a;
  a.theta = sd.theta;
  a.mom = sd.mom;
  a.gwp = sd.ws ? sd.ws + pl.gwp_off : nullptr;
  a.mass = sd.mass;
  a.step = sd.step;
  a.w_total = (int32_t)pl.w_total;
  a.n_rt = pl.n_row_tiles;
  a.n_rt_pad = pl.n_rt_pad;
  a.n_layers = pl.n_layers;
  for (int l = 0; l < DGPRF_MAX_LAYERS; ++l) {
    a.lo[l] = l < pl.n_layers ? (int32_t)pl.w_off[l] : INT32_MAX;
    a.hi[l] = l < pl.n_layers ? (int32_t)(pl.w_off[l] + (int64_t)pl.P[l] * pl.n_gp[l]) : 0;
  }
  a.seed = sd.seed;
  a.ws_cs = pl.ws_chain;
  a.step_offset = sd.step_offset;
  a.ud = ud;
  a.grad_in = grad_in;
  a.grad_out = sd.grad_out;
  a.grad_cs = pl.w_total + (sd.full_bayes ? pl.hyp_total : 0);
  a.gather_next = gather_next && sd.bd.mode == DGPRF_BATCH_EPOCH ? 1 : 0;
  a.B = pl.batch;
  a.d_in = pl.d_in;
  a.yb_cols = pl.yb_cols;
  a.bd = sd.bd;
  a.xb = sd.ws ? sd.ws + pl.xb_off : nullptr;
  a.yb = sd.ws ? sd.ws + pl.yb_off : nullptr;
  const int64_t quads = pl.w_total / 4;
  a.upd_blocks = (int)((quads + UPD_THREADS - 1) / UPD_THREADS);
  const bool gin = grad_in != nullptr, gonly = ud.grad_only != 0;
  const bool fb = sd.full_bayes && !gin;
  // full_bayesian=True: hyper workgroups first (per layer ceil(d R / HYP_EPB) for the Omega
  // rebuild, one in gradient-only mode), then the lik_log_var workgroup
  a.hyp_blocks = 0;
  a.pad_h = 0;
  std::memset(&a.hk, 0, sizeof(a.hk));
  size_t lds = 0;
  if (fb) {
    HypK& k = a.hk;
    k.hyp = sd.hyp;
    k.hmom = sd.hmom;
    k.hmass = sd.hmass;
    k.z = sd.z;
    k.omega = sd.omega;
    k.der = sd.der;
    k.ws = sd.ws;
    k.hyp_cs = sd.hyp_cs;
    k.om_cs = sd.om_cs;
    k.der_cs = sd.der_cs;
    k.hyp_total = pl.hyp_total;
    k.cnt_off = pl.hpl_off + pl.n_rt_pad;
    k.flags = pl.hyp_flags;
    k.likelihood = pl.likelihood;
    int nb_total = 0, hsmax = 4;
    for (int l = 0; l < pl.n_layers; ++l) {
      const int64_t n_el = (int64_t)pl.d[l] * pl.n_rf[l];
      const int nb = gonly ? 1 : (int)((n_el + HYP_EPB - 1) / HYP_EPB);
      k.d[l] = pl.d[l];
      k.R[l] = pl.n_rf[l];
      k.kind[l] = pl.kind[l];
      k.ard[l] = pl.ard[l];
      k.ns[l] = pl.ns[l];
      k.nb[l] = nb < 1 ? 1 : nb;
      k.b0[l] = nb_total;
      nb_total += k.nb[l];
      k.lis_off[l] = pl.lis_off[l];
      k.mean_off[l] = pl.mean_off[l];
      k.om_off[l] = pl.omega_off[l];
      k.hpp_off[l] = pl.hpp_off[l];
      hsmax = max(hsmax, round4(2 * pl.d[l] + 1));
      if (n_el >= (int64_t)1 << 29 || (int64_t)pl.n_rt_pad * NSM * round4(2 * pl.d[l] + 1) >= (int64_t)1 << 29)
        return hipErrorInvalidValue;  // 32-bit buffer offsets
    }
    k.hpl_off = pl.hpl_off;
    k.n_blocks = nb_total + 1;
    a.hyp_blocks = k.n_blocks;
    lds = (size_t)(5 * hsmax + max(4 * UPD_THREADS, hsmax) + UPD_THREADS + 4) * sizeof(float);
  }
  const int64_t gblocks = !a.gather_next ? 0 : (pl.d_in > GATHER_WIDE ? pl.batch
                                                    : (pl.batch + UPD_THREADS - 1) / UPD_THREADS);
  const int64_t blocks = a.hyp_blocks + a.upd_blocks + gblocks;
  dim3 grid((unsigned)blocks, pl.n_chains);
  const bool xi = ud.xi != nullptr || ud.xi_resample != nullptr ||
                  (fb && (ud.xi_hyp != nullptr || ud.xi_hyp_resample != nullptr));
  const bool cyc = ud.schedule == DGPRF_SCHED_CYCLICAL;
  const int sel = (gin ? 8 : 0) | (gonly ? 4 : 0) | (xi ? 2 : 0) | (cyc ? 1 : 0);
#define DGPRF_UPD_CASE(S)                                                                     \
  case S:                                                                                    \
    if (lds > 65536)                                                                         \
      dgprf::set_lds_limit(                                                                  \
          (const void*)k_step_update<(S & 8) != 0, (S & 4) != 0, (S & 2) != 0, (S & 1) != 0>, lds); \
    hipLaunchKernelGGL((k_step_update<(S & 8) != 0, (S & 4) != 0, (S & 2) != 0, (S & 1) != 0>), \
                       grid, dim3(UPD_THREADS), lds, s, a);                                  \
    break;
  switch (sel) {
    DGPRF_UPD_CASE(0) DGPRF_UPD_CASE(1) DGPRF_UPD_CASE(2) DGPRF_UPD_CASE(3)
    DGPRF_UPD_CASE(4) DGPRF_UPD_CASE(5) DGPRF_UPD_CASE(6) DGPRF_UPD_CASE(7)
    DGPRF_UPD_CASE(8) DGPRF_UPD_CASE(9) DGPRF_UPD_CASE(10) DGPRF_UPD_CASE(11)
    DGPRF_UPD_CASE(12) DGPRF_UPD_CASE(13) DGPRF_UPD_CASE(14) DGPRF_UPD_CASE(15)
  }
#undef DGPRF_UPD_CASE
  return hipGetLastError();
}


hipError_t launch_agemm(const float* X, int64_t n, int ld, int d, const float* om, int R,
                        float* aout, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (n <= INT32_MAX && blas_agemm(X, n, ld, d, om, R, aout, 1, 0, 0, 0, s)) return hipSuccess;
  if (n > INT32_MAX || (int64_t)n * ld >= ((int64_t)1 << 29) || (int64_t)d * R >= ((int64_t)1 << 29))
    return hipErrorInvalidValue;  // 32-bit buffer offsets
  AgemmK g;
  g.xrows = X;
  g.om = om;
  g.aout = aout;
  g.xrow_cs = g.om_cs = g.ws_cs = 0;
  g.B = (int32_t)n;
  g.d = d;
  g.R = R;
  g.d_in = ld;
  dim3 grid((unsigned)((R + 63) / 64), (unsigned)((n + 31) / 32), 1);
  hipLaunchKernelGGL(k_step_agemm, grid, dim3(256), 0, s, g);
  return hipGetLastError();
}

hipError_t launch_gather(const dgprf_plan_t& pl, const StepDev& sd, hipStream_t s) {
  if (sd.bd.mode == DGPRF_BATCH_DIRECT) return hipSuccess;
  GatherK a;
  a.bd = sd.bd;
  a.step = sd.step;
  a.xb = sd.ws + (sd.xb_sel ? pl.xb_alt_off : pl.xb_off);
  a.yb = sd.ws + (sd.xb_sel ? pl.yb_alt_off : pl.yb_off);
  a.ws_cs = pl.ws_chain;
  a.B = pl.batch;
  a.d_in = pl.d_in;
  a.yb_cols = pl.yb_cols;
  a.step_offset = sd.step_offset;
  const int rows_per_block = pl.d_in > GATHER_WIDE ? 4 : 256;
  dim3 grid((unsigned)((pl.batch + rows_per_block - 1) / rows_per_block), pl.n_chains);
  hipLaunchKernelGGL(k_gather, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_fresh_omega(const dgprf_plan_t& pl, const StepDev& sd, hipStream_t s) {
  if (!sd.hyp) return hipErrorInvalidValue;
  const int64_t quads = (pl.omega_total + 3) / 4;
  dim3 grid((unsigned)((quads + 255) / 256), pl.n_chains);
  hipLaunchKernelGGL(k_fresh_omega, grid, dim3(256), 0, s, pl, sd.hyp, sd.ws, sd.step, sd.seed,
                     sd.step_offset);
  return hipGetLastError();
}

hipError_t launch_advance(int64_t* step, int64_t by, hipStream_t s) {
  hipLaunchKernelGGL(k_advance, dim3(1), dim3(64), 0, s, step, by);
  return hipGetLastError();
}

}  // namespace dgprf
