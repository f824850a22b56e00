// k_vjp2, the packed-pair reverse mode of the narrow flows (cnf_vjp.hip
// describes the algorithm): kernel template and the types its instantiation
// tables share.  Included by cnf_vjp.hip (dispatch) and the three
// cnf_vjp2_*.hip translation units that instantiate it, five shapes each, so
// the library's slowest compile runs in parallel.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "cnf_internal.h"
#include "cnf_valu_common.h"
#include "cnf_sgpr_common.h"
#include "cnf_valu_io.h"

namespace cnf {

struct VArgs2 {
  const float* x;
  const int64_t* y;
  const float* gz;
  const float* gz_all;
  const float* gld;
  float* dx;
  float* partials;
  float* stash;  // [L][B][D/2] transformed-half layer inputs, (row 2i, row 2i+1) interleaved
  int64_t B;
  int L, kind;
  float det, grad_scale;
  int P, PS;
};

using VFn2 = void (*)(const float*, const int32_t*, const int32_t*, const int32_t*, VArgs2);

struct V2Entry {
  int D, H1, H2;
  VFn2 fn[2][2][2];  // [nets - 1][loss][perm]
};

// instantiation tables (cnf_vjp2_a/b/c.hip)
extern const V2Entry kV2PartA[];
extern const V2Entry kV2PartB[];
extern const V2Entry kV2PartC[];
extern const int kV2PartANum, kV2PartBNum, kV2PartCNum;

namespace v2 {
namespace {

using namespace valu;

typedef float floatx4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

constexpr float kEps = 1e-7f;  // calibrators.py:289

// ===========================================================================
// k_vjp2: reverse mode on packed row pairs (two rows per lane, v_pk_fma_f32)
// with the weights as SGPR operands (the plain packed-SGPR region), for the
// narrow shapes whose conditioner gradient stacks fit one 16x16 MFMA tile
// (GS = H1 + H2 + D/2 <= 16, HS = D - D/2 + H1 + H2 + 1 <= 16) and L <= 8.
//
// One wave per block walks tiles of 128 rows (grid-strided):
//   forward   the L layers, each layer's transformed-half input x_T stashed
//             in the workspace (HBM scratch, written and re-read by the same
//             wave within the tile: L2-resident in practice);
//   seed      the loss gradient (or gz / gld / gz_all of a generic VJP);
//   backward  per layer, last to first: undo flip / perm (renaming), recompute
//             both conditioners on the conditioning half, take the layer's
//             input x_T from the stash (recovering it as (z_T - t) exp(-s)
//             loses the reference's precision once |s| is large), back-
//             propagate through the affine update
//             and both MLPs (transposed products on SGPR weights);
//   dW        each net's G = [g_a1, g_a2, g_out] and H = [c, h1, h2, 1] go
//             through a 16 KB LDS stage 64 rows at a time and are folded into a
//             16x16 accumulator by v_mfma_f32_16x16x4f32 with the rows as K;
//             the accumulators of all (layer, net) live in registers for the
//             wave's whole run and are written once, as this wave's partial.
// Partials are summed in wave order by k_reduce_cols (deterministic).
// ===========================================================================
template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

constexpr int kV2TR = 128;   // rows per wave tile (lane l: rows 2l, 2l+1)
#ifndef CNF_V2_LMAX
#define CNF_V2_LMAX 8
#endif
constexpr int kV2LMax = CNF_V2_LMAX;  // layers the register accumulators hold
constexpr int kV2SS = 68;    // stage row stride in floats (64 rows + pad, 16-B aligned)



// widx: W[o][k] in the packed row layout [w_o0, b_o, w_o1 .. ] at stride S
template <int S>
__device__ __forceinline__ constexpr int widx(int o, int k) { return o * S + (k == 0 ? 0 : 1 + k); }

// y[o] = b[o] + sum_k W[o][k] x[k], o < NOUT (plain weights; input-major chains)
template <int NIN, int NOUT, int S, bool RELU, int NC>
__device__ __forceinline__ void vlin(const SW<NC>& w, const f2* x, f2* y) {
  f2 a[NOUT];
#pragma unroll
  for (int o = 0; o < NOUT; ++o) a[o] = fma_wb(w.pair(o * S), x[0]);
#pragma unroll
  for (int k = 1; k < NIN; ++k)
#pragma unroll
    for (int o = 0; o < NOUT; ++o) a[o] = fma_ws(w, widx<S>(o, k), x[k], a[o]);
#pragma unroll
  for (int o = 0; o < NOUT; ++o) y[o] = RELU ? maxT(a[o], splat(0.f, f2{})) : a[o];
}

// gacc[k] += sum_o W[o][k] gout[o] (the first Linear's input gradient goes
// straight into the running d/dc of the layer: no separate sum and add)
template <int NIN, int NOUT, int S, int NC>
__device__ __forceinline__ void vlin_t_acc(const SW<NC>& w, const f2* gout, f2* gacc) {
#pragma unroll
  for (int o = 0; o < NOUT; ++o)
#pragma unroll
    for (int k = 0; k < NIN; ++k) gacc[k] = fma_ws(w, widx<S>(o, k), gout[o], gacc[k]);
}

// gin[k] = sum_o W[o][k] gout[o], k < NIN, o < NOUT
template <int NIN, int NOUT, int S, int NC>
__device__ __forceinline__ void vlin_t(const SW<NC>& w, const f2* gout, f2* gin) {
#pragma unroll
  for (int k = 0; k < NIN; ++k) gin[k] = mul_ws(w, widx<S>(0, k), gout[0]);
#pragma unroll
  for (int o = 1; o < NOUT; ++o)
#pragma unroll
    for (int k = 0; k < NIN; ++k) gin[k] = fma_ws(w, widx<S>(o, k), gout[o], gin[k]);
}

// One net's activations on the conditioning half c (plain weights): h1, h2, out.
// Two SGPR buffers in turn: each Linear's block is issued before the previous
// Linear's FMAs (sready / sissue, cnf_sgpr_common.h), so only the net's first
// load waits its full latency.
template <class S, int NC>
__device__ __forceinline__ void vnet_fwd(const float* wn, const f2* c, f2* h1, f2* h2, f2* out) {
  SW<NC> A, Bw;
  sissue(A, wn);
  if constexpr (S::NL == 1) {
    sready();
    vlin<S::nin(0), S::nout(0), S::stride(0), false>(A, c, out);
  } else if constexpr (S::NL == 2) {
    sready();
    sissue(Bw, wn + S::off(1));
    vlin<S::nin(0), S::nout(0), S::stride(0), true>(A, c, h1);
    sready();
    vlin<S::nin(1), S::nout(1), S::stride(1), false>(Bw, h1, out);
  } else {
    sready();
    sissue(Bw, wn + S::off(1));
    vlin<S::nin(0), S::nout(0), S::stride(0), true>(A, c, h1);
    sready();
    sissue(A, wn + S::off(2));
    vlin<S::nin(1), S::nout(1), S::stride(1), true>(Bw, h1, h2);
    sready();
    vlin<S::nin(2), S::nout(2), S::stride(2), false>(A, h2, out);
  }
}

// The same net on the SCALED packed region (cnf_sgpr.hip's layout: hidden
// Linears x 2^-64 with the next Linear's input columns x 2^64, the s-net's last
// Linear x log2 e): ReLU is the clamp bit of each hidden neuron's last FMA, so
// h1, h2 come out as h' = 2^-64 h (exact: powers of two) and the s-net's output
// as s' = log2(e) s.  Saves the two unpacked v_max (plus their canonicalising
// copies) per pair and hidden neuron of the plain form.
template <int NIN, int NOUT, int S, bool CLAMP, int NC>
__device__ __forceinline__ void vlin_sp(const SW<NC>& w, const f2* x, f2* y) {
  f2 a[NOUT];
#pragma unroll
  for (int o = 0; o < NOUT; ++o)
    a[o] = (CLAMP && NIN == 1) ? fma_wb_clamp(w.pair(o * S), x[0]) : fma_wb(w.pair(o * S), x[0]);
#pragma unroll
  for (int k = 1; k < NIN; ++k)
#pragma unroll
    for (int o = 0; o < NOUT; ++o)
      a[o] = (CLAMP && k == NIN - 1) ? fma_ws_clamp(w, widx<S>(o, k), x[k], a[o])
                                     : fma_ws(w, widx<S>(o, k), x[k], a[o]);
#pragma unroll
  for (int o = 0; o < NOUT; ++o) y[o] = a[o];
}
template <class S, int NC>
__device__ __forceinline__ void vnet_fwd_sp(const float* wn, const f2* c, f2* h1, f2* h2, f2* out) {
  SW<NC> A, Bw;
  sissue(A, wn);
  if constexpr (S::NL == 1) {
    sready();
    vlin_sp<S::nin(0), S::nout(0), S::stride(0), false>(A, c, out);
  } else if constexpr (S::NL == 2) {
    sready();
    sissue(Bw, wn + S::off(1));
    vlin_sp<S::nin(0), S::nout(0), S::stride(0), true>(A, c, h1);
    sready();
    vlin_sp<S::nin(1), S::nout(1), S::stride(1), false>(Bw, h1, out);
  } else {
    sready();
    sissue(Bw, wn + S::off(1));
    vlin_sp<S::nin(0), S::nout(0), S::stride(0), true>(A, c, h1);
    sready();
    sissue(A, wn + S::off(2));
    vlin_sp<S::nin(1), S::nout(1), S::stride(1), true>(Bw, h1, h2);
    sready();
    vlin_sp<S::nin(2), S::nout(2), S::stride(2), false>(A, h2, out);
  }
}

// relu' from the recomputed activation h' = 2^-64 relu(pre) (the clamp-ReLU
// output of vnet_fwd_sp: in [0, 1], 0 for a NaN pre-activation), as torch's
// threshold_backward: drops g where h' = 0 and keeps it otherwise.
// Default (2): clamp((h' 2^127) 2^127) * g, three packed ops per pair, no VCC
// (the compare-and-select form, 0, costs two v_cmp + two v_cndmask per pair
// plus the VCC hazard's wait states): 0.1765 -> 0.1750 ms per cfg2 step,
// gradients bitwise unchanged.
#ifndef CNF_V2_CLAMP_MASK
#define CNF_V2_CLAMP_MASK 2
#endif
#if CNF_V2_CLAMP_MASK == 0
__device__ __forceinline__ f2 relu_mask(f2 g, f2 h) {
  return f2{h.x <= 0.f ? 0.f : g.x, h.y <= 0.f ? 0.f : g.y};
}
#elif CNF_V2_CLAMP_MASK == 1
// A/B: the mask as clamp(h' 2^127) (packed; NaN clamps to 0) times g -- exact
// for h' = 2^-64 h >= 2^-127, i.e. every pre-activation above 2^-63
__device__ __forceinline__ f2 relu_mask(f2 g, f2 h) {
  f2 m;
  asm("v_pk_mul_f32 %0, %1, %2 clamp" : "=v"(m) : "v"(h), "s"(splat(0x1p127f, f2{})));
  return g * m;
}
#else
// clamp((h' 2^127) 2^127) times g -- exact for every h' > 0 (f32
// denormals are kept: the smallest, 2^-149, maps to 2^105 before the clamp);
// h' is the clamp-ReLU output, so h' in [0, 1] and 0 for a NaN pre-activation
__device__ __forceinline__ f2 relu_mask(f2 g, f2 h) {
  f2 m, u;
  const f2 k = splat(0x1p127f, f2{});
  asm("v_pk_mul_f32 %0, %1, %2" : "=v"(u) : "v"(h), "s"(k));
  asm("v_pk_mul_f32 %0, %1, %2 clamp" : "=v"(m) : "v"(u), "s"(k));
  return g * m;
}
#endif

// Back-propagate one net: gout (d/d out) -> adds d/dc into gc and leaves the
// gradient stack G = [g_a1, g_a2, gout] (pre-activation gradients).
template <class S, int NC>
__device__ __forceinline__ void vnet_bwd(const float* wn, const f2* h1, const f2* h2,
                                         const f2* gout, f2* gc, f2* G) {
  constexpr int H1 = S::NL >= 2 ? S::nout(0) : 0, H2 = S::NL == 3 ? S::nout(1) : 0;
  constexpr int DT = S::DT, DC = S::DC;
  SW<NC> A, Bw;
  if constexpr (S::NL == 1) {
    sissue(A, wn);
    sready();
    vlin_t_acc<DC, DT, S::stride(0)>(A, gout, gc);
  } else if constexpr (S::NL == 2) {
    f2 g1[H1];
    sissue(A, wn + S::off(1));
    sready();
    sissue(Bw, wn);
    vlin_t<H1, DT, S::stride(1)>(A, gout, g1);
#pragma unroll
    for (int m = 0; m < H1; ++m) G[m] = g1[m] = relu_mask(g1[m], h1[m]);
    sready();
    vlin_t_acc<DC, H1, S::stride(0)>(Bw, g1, gc);
  } else {
    f2 g2[H2], g1[H1];
    sissue(A, wn + S::off(2));
    sready();
    sissue(Bw, wn + S::off(1));
    vlin_t<H2, DT, S::stride(2)>(A, gout, g2);
#pragma unroll
    for (int m = 0; m < H2; ++m) G[H1 + m] = g2[m] = relu_mask(g2[m], h2[m]);
    sready();
    sissue(A, wn);
    vlin_t<H1, H2, S::stride(1)>(Bw, g2, g1);
#pragma unroll
    for (int m = 0; m < H1; ++m) G[m] = g1[m] = relu_mask(g1[m], h1[m]);
    sready();
    vlin_t_acc<DC, H1, S::stride(0)>(A, g1, gc);
  }
#pragma unroll
  for (int j = 0; j < DT; ++j) G[H1 + H2 + j] = gout[j];
}

// Fold G^T H of this tile's 128 rows (GS x HS <= 16 x 16) into acc: the stage
// holds 64 rows at a time ([feature][row], G features 0..15 then H 16..31);
// lane l feeds MFMA step ks with feature l%16 of row (l/16)*16 + ks, so its
// operands for all 16 steps are 16 contiguous floats (4 ds_read_b128).
template <int GS, int HS>
__device__ __forceinline__ floatx4 wgrad_tile(float* st, const f2* G, const f2* H, int lane,
                                              floatx4 acc) {
#pragma unroll
  for (int ch = 0; ch < 2; ++ch) {
    wave_sync();  // the previous reads of the stage are done
#pragma unroll
    for (int f = 0; f < GS; ++f) st[f * kV2SS + lane] = ch ? G[f].y : G[f].x;
#pragma unroll
    for (int f = 0; f < HS; ++f) st[(16 + f) * kV2SS + lane] = ch ? H[f].y : H[f].x;
    wave_sync();
    const float4* ga = reinterpret_cast<const float4*>(st + (lane & 15) * kV2SS + (lane >> 4) * 16);
    const float4* hb =
        reinterpret_cast<const float4*>(st + (16 + (lane & 15)) * kV2SS + (lane >> 4) * 16);
    float4 A[4], Bv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      A[q] = ga[q];
      Bv[q] = hb[q];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A[q].x, Bv[q].x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A[q].y, Bv[q].y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A[q].z, Bv[q].z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A[q].w, Bv[q].w, acc, 0, 0, 0);
    }
  }
  return acc;
}

// A/B: the x_T stash feature-major [L][DT][Bp] (whole-line stores) and
// streaming (nt) stash traffic.  cfg2 step: row-major 0.1565-0.1577 ms,
// feature-major 0.1581-0.1588, + nt stores 0.1647-0.1671, + nt loads too
// 0.1643-0.1658 -- the stash is re-read one tile later and partly hits L2.
#ifndef CNF_V2_STASH_FM
#define CNF_V2_STASH_FM 0
#endif
#ifndef CNF_V2_STASH_NT
#define CNF_V2_STASH_NT 0  // bit 0: streaming stash stores, bit 1: streaming stash loads
#endif
#ifndef CNF_V2_HLATE
#define CNF_V2_HLATE 1  // the dW stack's 2^64 on h' applied once per wave (below)
#endif
#ifndef CNF_V2_TLATE
#define CNF_V2_TLATE 0  // A/B: the t-net recompute after the s-net's backward step
#endif
#ifndef CNF_V2_WPS
#define CNF_V2_WPS 2  // waves per SIMD the register budget is held to
#endif

// parameter p (state_dict order of one layer) -> (G row i, H column j) of its
// gradient in the (layer, net) tile, or -1 when the gradient is zero by the mask
// (the transformed-half inputs of the first Linear, the conditioning-half
// outputs of the last).  Returns the net index through *net.
template <int D, int H1, int H2, int NETS>
__device__ __forceinline__ int param_cell(int r, int* net) {
  using S = SP<D, H1, H2>;
  constexpr int DT = S::DT, DC = S::DC, NL = S::NL;
  constexpr int U[4] = {D, H1 ? H1 : D, H2 ? H2 : D, D};
  constexpr int NFN = H1 == 0 ? D * D + D : (H2 == 0 ? H1 * D + H1 + D * H1 + D
                                                      : H1 * D + H1 + H2 * H1 + H2 + D * H2 + D);
  constexpr int HS = DC + H1 + H2 + 1;
  *net = r / NFN;
  r -= *net * NFN;
  int gofs = 0, hofs = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int nin = U[i], nout = i == NL - 1 ? D : U[i + 1];
    const bool first = i == 0, last = i == NL - 1;
    const int nout_eff = last ? DT : nout, nin_eff = first ? DC : nin;
    if (r < nout * nin) {
      const int o = r / nin, col = r - o * nin;
      const int kk = first ? col - DT : col;
      return (o < nout_eff && kk >= 0 && kk < nin_eff) ? (gofs + o) * 16 + hofs + kk : -1;
    }
    r -= nout * nin;
    if (r < nout) return r < nout_eff ? (gofs + r) * 16 + HS - 1 : -1;
    r -= nout;
    gofs += nout_eff;
    hofs += nin_eff;
  }
  return -1;
}

// accumulator cell (G row i, H column j) -> offset of its parameter in the
// net's state_dict block, or -1 (a cell of the dense tile with no parameter)
template <int D, int H1, int H2>
__device__ __forceinline__ int cell_param(int i, int j) {
  using S = SP<D, H1, H2>;
  constexpr int DT = S::DT, DC = S::DC, NL = S::NL;
  constexpr int U[4] = {D, H1 ? H1 : D, H2 ? H2 : D, D};
  constexpr int HS = DC + H1 + H2 + 1;
  int gofs = 0, hofs = 0, woff = 0;
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const int nin = U[k], nout = k == NL - 1 ? D : U[k + 1];
    const bool first = k == 0, last = k == NL - 1;
    const int nout_eff = last ? DT : nout, nin_eff = first ? DC : nin, in_off = first ? DT : 0;
    if (i >= gofs && i < gofs + nout_eff) {
      const int o = i - gofs;
      if (j == HS - 1) return woff + nout * nin + o;
      if (j >= hofs && j < hofs + nin_eff) return woff + o * nin + in_off + (j - hofs);
      return -1;
    }
    woff += nout * nin + nout;
    gofs += nout_eff;
    hofs += nin_eff;
  }
  return -1;
}

template <int D, int H1, int H2, int NETS, bool LOSS, bool PERM>
__global__ __launch_bounds__(64, CNF_V2_WPS) void k_vjp2(const float* __restrict__ W,
                                                const int32_t* __restrict__ fq,
                                                const int32_t* __restrict__ iq,
                                                const int32_t* __restrict__ lflag, VArgs2 a) {
  using S = SP<D, H1, H2>;
  constexpr int DT = S::DT, DC = S::DC, NC = S::NC;
  constexpr int LF = NETS * S::NF;
  constexpr int GS = H1 + H2 + DT, HS = DC + H1 + H2 + 1;
  static_assert(GS <= 16 && HS <= 16, "gradient stacks must fit one 16x16 MFMA tile");
  constexpr int TF = kV2TR * D;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* tile = smem;        // [TF] input rows
  float* st = smem + TF;     // [32][kV2SS] G / H stage
  constexpr int kStage = 32 * kV2SS;
  const int lane = threadIdx.x;
  const int64_t B = a.B;
  const int64_t Bp = (B + 1) & ~(int64_t)1;  // stash rows per feature (8-B aligned pairs)
  const int L = a.L;
  const int ntiles = (int)((B + kV2TR - 1) / kV2TR);
  const f2 zero = splat(0.f, f2{});
  constexpr float kLN2 = 0.69314718055994531f, kL2E = 1.4426950408889634f;
  // the scaled packed region (forward sweep and recompute) sits right before
  // the plain one (back-propagation): cnf_prepare's sp_region / vp_region
  const float* __restrict__ Wsp = W - (int64_t)L * LF;
  constexpr float kTwo64 = 0x1p64f;  // h = 2^64 h' (exact)
#if CNF_V2_HLATE
  // H takes h' itself: the hidden columns of the accumulators are 2^-64 times
  // the gradient and get the 2^64 once, when the wave writes its partial (a
  // power-of-two scale commutes with every rounding of the sum until the
  // products fall below 2^-126, i.e. |g h| < 2^-62)
  constexpr float kHs = 1.f;
#else
  constexpr float kHs = kTwo64;
#endif
  floatx4 acc[kV2LMax][NETS];
#pragma unroll
  for (int l = 0; l < kV2LMax; ++l)
#pragma unroll
    for (int n = 0; n < NETS; ++n) acc[l][n] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int i = lane; i < kStage; i += 64) st[i] = 0.f;
  float lt0 = 0.f, lt1 = 0.f, lt2 = 0.f;

  for (int tix = blockIdx.x; tix < ntiles; tix += gridDim.x) {
    const int64_t row0 = (int64_t)tix * kV2TR;
    const int64_t r = row0 + 2 * lane;
    const int nr = r >= B ? 0 : (r + 1 >= B ? 1 : 2);
    const bool full = row0 + kV2TR <= B;  // wave-uniform: every lane holds two rows
    // ---- rows in: one tile through LDS (full tiles: 16-B loads) ----
    f2 v[D];
    if (row0 + kV2TR <= B) {
      wave_sync();
      const float4* s4 = reinterpret_cast<const float4*>(a.x + row0 * D);
      float4* d4 = reinterpret_cast<float4*>(tile);
      for (int i = lane; i < TF / 4; i += 64) d4[i] = s4[i];
      wave_sync();
      f2 vv[1][D];
      read_pairs<D, 1>(tile, lane, vv);
#pragma unroll
      for (int k = 0; k < D; ++k) v[k] = vv[0][k];
    } else {
#pragma unroll
      for (int k = 0; k < D; ++k)
        v[k] = f2{nr > 0 ? a.x[r * D + k] : 0.f, nr > 1 ? a.x[(r + 1) * D + k] : 0.f};
    }
    uint32_t lab = 0;
    if constexpr (LOSS) lab = load_labels<D, 1>(a.y + r, nr, false);

    // ---- forward sweep (plain weights, nothing stashed) ----
    f2 ld = zero;
    auto fwd = [&](auto O_, int l) __attribute__((always_inline)) {
      constexpr bool O = decltype(O_)::value;
      f2 c[DC];
#pragma unroll
      for (int k = 0; k < DC; ++k) c[k] = v[R<D, O>(DT + k)];
      f2 h1[H1 ? H1 : 1], h2[H2 ? H2 : 1], t[DT], sv[DT];
      {  // x_T of this layer, rows r, r+1
#if CNF_V2_STASH_FM
        // feature-major [L][DT][Bp]: each 8-B store instruction writes 512
        // contiguous bytes (whole lines), streamed past L2 (STASH_NT bit 0)
        float* sp = a.stash + (int64_t)l * DT * Bp + r;
        if (full) {
#pragma unroll
          for (int j = 0; j < DT; ++j) {
            if (CNF_V2_STASH_NT & 1)
              __builtin_nontemporal_store(v[R<D, O>(j)], reinterpret_cast<f2*>(sp + j * Bp));
            else
              *reinterpret_cast<f2*>(sp + j * Bp) = v[R<D, O>(j)];
          }
        } else {
#pragma unroll
          for (int j = 0; j < DT; ++j) {
            if (nr > 0) sp[j * Bp] = v[R<D, O>(j)].x;
            if (nr > 1) sp[j * Bp + 1] = v[R<D, O>(j)].y;
          }
        }
#else
        // row-major [L][B][DT]: 2*DT contiguous floats as (row r, row r+1)
        // pairs (8-B stores: the lane's slot starts 8-B aligned)
        float* sp = a.stash + ((int64_t)l * B + r) * DT;
        if (full) {
#pragma unroll
          for (int j = 0; j < DT; ++j) reinterpret_cast<f2*>(sp)[j] = v[R<D, O>(j)];
        } else {
#pragma unroll
          for (int j = 0; j < DT; ++j) {
            if (nr > 0) sp[2 * j] = v[R<D, O>(j)].x;
            if (nr > 1) sp[2 * j + 1] = v[R<D, O>(j)].y;
          }
        }
#endif
      }
      const float* ws = Wsp + (int64_t)l * LF;
      vnet_fwd_sp<S, NC>(ws + (NETS == 2 ? S::NF : 0), c, h1, h2, t);
      if constexpr (NETS == 2) vnet_fwd_sp<S, NC>(ws, c, h1, h2, sv);  // sv = log2(e) s
#pragma unroll
      for (int j = 0; j < DT; ++j) {
        f2& x = v[R<D, O>(j)];
        if constexpr (NETS == 2) {
          x = fmaV(x, exp2T(sv[j]), t[j]);
          ld += sv[j];
        } else {
          x += t[j];
        }
      }
      if constexpr (PERM) {
        if (lflag[l] & kFlagPerm) permute<D, O>(v, fq + l * D);
      }
    };
    int l = 0;
    for (; l + 1 < L; l += 2) {
      fwd(std::false_type{}, l);
      fwd(std::true_type{}, l + 1);
    }
    const bool oddL = l < L;
    if (oddL) fwd(std::false_type{}, l);
    if constexpr (NETS == 2) ld = ld * splat(kLN2, f2{});  // ln2 sum(s')

    // ---- upstream gradient at z_L (orientation L & 1) ----
    f2 g[D];
    f2 gld = zero;
    auto seed = [&](auto O_) __attribute__((always_inline)) {
      constexpr bool O = decltype(O_)::value;
#ifndef CNF_V2_SCALAR_SEED
      if constexpr (LOSS) {
        // Both rows as packed pairs (k_sgpr's pair_loss form): the max, the
        // exponentials e_j = exp(z_j - m) (kept: p_j = e_j / se, no second
        // exp pass), the sum, and the gradient scale(coef) * p_j.  The rows'
        // z[y] come from the wave's LDS tile (the lane's two rows at tile
        // [0, D) and [D, 2D), as the input was read), and the one-hot
        // subtraction g_y -= scale * coef is an LDS add at that slot before
        // the pairs are read back -- no per-row select trees.
        typedef __attribute__((address_space(3))) float lds_f;
        const uint32_t tb = (uint32_t)(uintptr_t)(lds_f*)(tile + 2 * D * lane);
        wave_sync();  // every lane's rows were read from the tile long ago
#pragma unroll
        for (int j = 0; j < D; ++j)
          asm volatile("ds_write2_b32 %0, %1, %2 offset0:%3 offset1:%4" ::"v"(tb),
                       "v"(v[R<D, O>(j)].x), "v"(v[R<D, O>(j)].y), "i"(j), "i"(D + j)
                       : "memory");
        const uint32_t b0 = lab & 0xffu, b1 = (lab >> 8) & 0xffu;
        const bool ok[2] = {b0 != 0xffu, b1 != 0xffu};
        const int yy[2] = {ok[0] ? (int)b0 : 0, ok[1] ? (int)b1 : 0};
        float zy[2];
        zy[0] = tile[2 * D * lane + yy[0]];
        zy[1] = tile[2 * D * lane + D + yy[1]];
        f2 m = v[R<D, O>(0)];
#pragma unroll
        for (int j = 1; j < D; ++j) m = maxT(m, v[R<D, O>(j)]);
        const f2 nm = m * splat(-kL2E, f2{});
        f2 e[D], se = zero;
#pragma unroll
        for (int j = 0; j < D; ++j) {
          e[j] = exp2T(fmaT(kL2E, v[R<D, O>(j)], nm));
          se += e[j];
        }
        f2 sc;  // grad_scale * coef / se per row
        float dy[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const float lse = m[q] + __builtin_amdgcn_logf(se[q]) * kLN2;
          const float lpy = zy[q] - lse;
          const bool valid = q < nr;
          const float ldq = NETS == 2 ? ld[q] : 0.f;
          float coef, ce_term, loss_row, gl;
          if (a.kind == CNF_LOSS_CAL) {  // -(log(softmax(z)[y] + 1e-7) + ld)
            const float py = __builtin_amdgcn_exp2f(lpy * kL2E);
            ce_term = -__builtin_amdgcn_logf(py + kEps) * kLN2;
            loss_row = ce_term - ldq;
            coef = py / (py + kEps);
            gl = -a.grad_scale;
          } else {                       // CE(z, y) - det * ld
            ce_term = -lpy;
            loss_row = ce_term - a.det * ldq;
            coef = 1.f;
            gl = -a.det * a.grad_scale;
          }
          if (!ok[q]) ce_term = loss_row = coef = __builtin_nanf("");
          if (!valid) coef = gl = 0.f;
          sc[q] = a.grad_scale * coef / se[q];
          dy[q] = -a.grad_scale * coef;
          gld[q] = gl;
          if (valid) {
            lt0 += loss_row;
            lt1 += ce_term;
            lt2 += ldq;
          }
        }
        // g_j = sc e_j, then g_y += dy: staged over the z rows (same slots)
#pragma unroll
        for (int j = 0; j < D; ++j) {
          const f2 gj = e[j] * sc;
          asm volatile("ds_write2_b32 %0, %1, %2 offset0:%3 offset1:%4" ::"v"(tb), "v"(gj.x),
                       "v"(gj.y), "i"(j), "i"(D + j)
                       : "memory");
        }
        asm volatile("ds_add_f32 %0, %1" ::"v"(tb + 4u * yy[0]), "v"(dy[0]) : "memory");
        asm volatile("ds_add_f32 %0, %1 offset:%2" ::"v"(tb + 4u * yy[1]), "v"(dy[1]), "i"(4 * D)
                     : "memory");
        {  // the reads and their wait in one asm statement (ds_read2_pairs)
          f2 o[D];
          ds_read2_pairs<D>(tb, o);
#pragma unroll
          for (int j = 0; j < D; ++j) g[R<D, O>(j)] = o[j];
        }
      } else
#endif
      if constexpr (LOSS) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          float z[D];
#pragma unroll
          for (int j = 0; j < D; ++j) z[j] = v[R<D, O>(j)][q];
          float m = z[0];
#pragma unroll
          for (int j = 1; j < D; ++j) m = fmaxf(m, z[j]);
          float se = 0.f;
#pragma unroll
          for (int j = 0; j < D; ++j) se += __builtin_amdgcn_exp2f((z[j] - m) * kL2E);
          const float lse = m + __builtin_amdgcn_logf(se) * kLN2;
          const uint32_t b = (lab >> (8 * q)) & 0xffu;
          const bool ok = b != 0xffu, valid = q < nr;
          const int yy = ok ? (int)b : 0;
          uint32_t zb[D];
#pragma unroll
          for (int j = 0; j < D; ++j) zb[j] = __float_as_uint(z[j]);
          const float lpy = __uint_as_float(sel_tree<D>(zb, yy, 0)) - lse;
          const float ldq = NETS == 2 ? ld[q] : 0.f;  // plain weights: ld = sum(s)
          float coef, ce_term, loss_row, gl;
          if (a.kind == CNF_LOSS_CAL) {  // -(log(softmax(z)[y] + 1e-7) + ld)
            const float py = __builtin_amdgcn_exp2f(lpy * kL2E);
            ce_term = -__builtin_amdgcn_logf(py + kEps) * kLN2;
            loss_row = ce_term - ldq;
            coef = py / (py + kEps);
            gl = -a.grad_scale;
          } else {                       // CE(z, y) - det * ld
            ce_term = -lpy;
            loss_row = ce_term - a.det * ldq;
            coef = 1.f;
            gl = -a.det * a.grad_scale;
          }
          if (!ok) ce_term = loss_row = coef = __builtin_nanf("");
          if (!valid) coef = gl = 0.f;
#pragma unroll
          for (int j = 0; j < D; ++j) {
            const float pj = __builtin_amdgcn_exp2f((z[j] - lse) * kL2E);
            g[R<D, O>(j)][q] = a.grad_scale * coef * (pj - (j == yy ? 1.f : 0.f));
          }
          gld[q] = gl;
          if (valid) {
            lt0 += loss_row;
            lt1 += ce_term;
            lt2 += ldq;
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < D; ++j)
          g[R<D, O>(j)] = f2{a.gz && nr > 0 ? a.gz[r * D + j] : 0.f,
                              a.gz && nr > 1 ? a.gz[(r + 1) * D + j] : 0.f};
        gld = f2{a.gld && nr > 0 ? a.gld[r] : 0.f, a.gld && nr > 1 ? a.gld[r + 1] : 0.f};
      }
    };
    if (oddL) seed(std::true_type{});
    else seed(std::false_type{});

    // ---- backward sweep ----
    // layer index compile-time (static_for below): the per-layer gradient
    // accumulators acc[l][net] stay in registers (a runtime-indexed select
    // over them was lowered to scratch)
    auto bwd = [&](auto LI) __attribute__((always_inline)) {
      constexpr int l = decltype(LI)::value;
      constexpr bool Oc = ((l + 1) & 1) != 0;  // orientation of z_l
      constexpr bool Oi = !Oc;
      if (!LOSS && a.gz_all) {  // (the loss entry points never pass gz_all)
#pragma unroll
        for (int j = 0; j < D; ++j)
          g[R<D, Oc>(j)] += f2{nr > 0 ? a.gz_all[((int64_t)l * B + r) * D + j] : 0.f,
                               nr > 1 ? a.gz_all[((int64_t)l * B + r + 1) * D + j] : 0.f};
      }
      if constexpr (PERM) {
        if (lflag[l] & kFlagPerm) {  // undo z[:, perm].flip(1): z_pre[i] = z_out[iq[i]]
          permute<D, Oc>(v, iq + l * D);
          permute<D, Oc>(g, iq + l * D);
        }
      }
      // the layer's weight offset laundered through an SGPR: left as a constant,
      // the compiler hoists all eight layers' 64-bit block addresses out of the
      // tile loop and spills them to VGPR lanes (v_readlane before every load)
      int lofs = l * LF;
      asm volatile("" : "+s"(lofs));
      const float* wl = W + lofs;
      f2 c[DC], gT[DT], gc[DC];
#pragma unroll
      for (int k = 0; k < DC; ++k) {
        c[k] = v[R<D, Oi>(DT + k)];
        gc[k] = zero;
      }
#pragma unroll
      for (int j = 0; j < DT; ++j) gT[j] = g[R<D, Oi>(j)];
      f2 xT[DT];
      {
#if CNF_V2_STASH_FM
        const float* sp = a.stash + (int64_t)l * DT * Bp + r;
        if (full) {
#pragma unroll
          for (int j = 0; j < DT; ++j) {
            if (CNF_V2_STASH_NT & 2)
              xT[j] = __builtin_nontemporal_load(reinterpret_cast<const f2*>(sp + j * Bp));
            else
              xT[j] = *reinterpret_cast<const f2*>(sp + j * Bp);
          }
        } else {
#pragma unroll
          for (int j = 0; j < DT; ++j)
            xT[j] = f2{nr > 0 ? sp[j * Bp] : 0.f, nr > 1 ? sp[j * Bp + 1] : 0.f};
        }
#else
        const float* sp = a.stash + ((int64_t)l * B + r) * DT;
        if (full) {
#pragma unroll
          for (int j = 0; j < DT; ++j) xT[j] = reinterpret_cast<const f2*>(sp)[j];
        } else {
#pragma unroll
          for (int j = 0; j < DT; ++j)
            xT[j] = f2{nr > 0 ? sp[2 * j] : 0.f, nr > 1 ? sp[2 * j + 1] : 0.f};
        }
#endif
      }
      // recompute on the scaled weights: th / sh are 2^-64 h (relu' reads
      // their sign; the weight-gradient stack H takes 2^64 times them)
      const float* ws = Wsp + lofs;
      f2 th1[H1 ? H1 : 1], th2[H2 ? H2 : 1], t[DT];
#if !CNF_V2_TLATE
      vnet_fwd_sp<S, NC>(ws + (NETS == 2 ? S::NF : 0), c, th1, th2, t);
#endif
      f2 H[HS];
#pragma unroll
      for (int k = 0; k < DC; ++k) H[k] = c[k];
      H[HS - 1] = splat(1.f, f2{});
      // invalid (padding) rows contribute nothing to the weight gradients
      const f2 keep = f2{nr > 0 ? 1.f : 0.f, nr > 1 ? 1.f : 0.f};
      if constexpr (NETS == 2) {
        f2 sh1[H1 ? H1 : 1], sh2[H2 ? H2 : 1], sv[DT];
        vnet_fwd_sp<S, NC>(ws, c, sh1, sh2, sv);  // sv = log2(e) s
        f2 gs[DT];
#pragma unroll
        for (int j = 0; j < DT; ++j) {
          const f2 e = exp2T(sv[j]);
          gs[j] = fmaV(gT[j] * xT[j], e, gld);  // z_T = x_T e^s + t, ld += s
          gT[j] = gT[j] * e;
        }
        f2 G[GS];
        vnet_bwd<S, NC>(wl, sh1, sh2, gs, gc, G);
        if (!full) {
#pragma unroll
          for (int f = 0; f < GS; ++f) G[f] *= keep;
        }
#pragma unroll
        for (int m = 0; m < H1; ++m) H[DC + m] = sh1[m] * splat(kHs, f2{});
#pragma unroll
        for (int m = 0; m < H2; ++m) H[DC + H1 + m] = sh2[m] * splat(kHs, f2{});
        acc[l][0] = wgrad_tile<GS, HS>(st, G, H, lane, acc[l][0]);
      }
      {  // t-net: d/dt = g_T (before the e^s scaling of the s-net branch)
#if CNF_V2_TLATE
        // recomputed only now: th1 / th2 are not live across the s-net's step
        vnet_fwd_sp<S, NC>(ws + (NETS == 2 ? S::NF : 0), c, th1, th2, t);
#endif
        f2 G[GS];
        f2 gt[DT];
#pragma unroll
        for (int j = 0; j < DT; ++j) gt[j] = g[R<D, Oi>(j)];
        vnet_bwd<S, NC>(wl + (NETS == 2 ? S::NF : 0), th1, th2, gt, gc, G);
        if (!full) {
#pragma unroll
          for (int f = 0; f < GS; ++f) G[f] *= keep;
        }
#pragma unroll
        for (int m = 0; m < H1; ++m) H[DC + m] = th1[m] * splat(kHs, f2{});
#pragma unroll
        for (int m = 0; m < H2; ++m) H[DC + H1 + m] = th2[m] * splat(kHs, f2{});
        acc[l][NETS - 1] = wgrad_tile<GS, HS>(st, G, H, lane, acc[l][NETS - 1]);
      }
#pragma unroll
      for (int j = 0; j < DT; ++j) {
        v[R<D, Oi>(j)] = xT[j];
        g[R<D, Oi>(j)] = gT[j];
      }
#pragma unroll
      for (int k = 0; k < DC; ++k) g[R<D, Oi>(DT + k)] += gc[k];
    };
    static_for<0, kV2LMax>([&](auto I) __attribute__((always_inline)) {
      constexpr int l = kV2LMax - 1 - decltype(I)::value;
      if (l < L) bwd(std::integral_constant<int, l>{});
    });
    if (a.dx) {
#pragma unroll
      for (int j = 0; j < D; ++j) {
        if (nr > 0) a.dx[r * D + j] = g[j].x;
        if (nr > 1) a.dx[(r + 1) * D + j] = g[j].y;
      }
    }
  }

  // ---- this wave's partial: parameter gradients (state_dict order) + loss sums ----
  float* out = a.partials + (int64_t)blockIdx.x * a.PS;
  const int P = a.P;
  constexpr int NFN = H1 == 0 ? D * D + D : (H2 == 0 ? H1 * D + H1 + D * H1 + D
                                                      : H1 * D + H1 + H2 * H1 + H2 + D * H2 + D);
  // zeros where the mask makes the gradient vanish: the same offsets in every
  // (layer, net) block, so the lane classifies its offsets lane + 64 k of one
  // block once (a param_cell per element of P was ~4 % of the launch's VALU)
  {
    constexpr int KB = (NFN + 63) / 64;
    bool zr[KB];
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      int n;
      const int rr = lane + 64 * k;
      zr[k] = rr < NFN && param_cell<D, H1, H2, 1>(rr, &n) < 0;
    }
    for (int blk = 0; blk < L * NETS; ++blk)
#pragma unroll
      for (int k = 0; k < KB; ++k)
        if (zr[k]) out[blk * NFN + lane + 64 * k] = 0.f;
  }
  // the lane's accumulator cells: C[i = 4 (lane/16) + e][j = lane % 16]
  const int j = lane & 15, i0 = 4 * (lane >> 4);
  const float hsc = (CNF_V2_HLATE && j >= DC && j < DC + H1 + H2) ? kTwo64 : 1.f;
  // the cells' offsets within a net's block: the same for every (layer, net),
  // mapped once (laundered, so the mapping is not re-derived per store) and
  // gathered into one exec mask
  int q[4];
  bool any = false;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    q[e] = cell_param<D, H1, H2>(i0 + e, j);
    asm volatile("" : "+v"(q[e]));
    any |= q[e] >= 0;
  }
  if (any) {
    static_for<0, kV2LMax>([&](auto I) __attribute__((always_inline)) {
      constexpr int l = decltype(I)::value;
      if (l >= L) return;
#pragma unroll
      for (int n = 0; n < NETS; ++n) {
        const floatx4 c4 = acc[l][n];
        // net n's parameters follow the layer's state_dict order: s-net first
        float* ob = out + l * NETS * NFN + n * NFN;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (q[e] >= 0) ob[q[e]] = c4[e] * hsc;
      }
    });
  }
  if constexpr (LOSS) {  // the wave's loss sums (DPP, into lane 63: cnf_valu_io.h)
    lt0 = wave_sum_dpp63(lt0);
    lt1 = wave_sum_dpp63(lt1);
    lt2 = wave_sum_dpp63(lt2);
    if (lane == 63) {
      out[P] = lt0;
      out[P + 1] = lt1;
      out[P + 2] = lt2;
    }
  }
}


}  // namespace
}  // namespace v2

#define CNF_V2N(D, H1, H2, N)                                                                  \
  {{v2::k_vjp2<D, H1, H2, N, false, false>, v2::k_vjp2<D, H1, H2, N, false, true>},          \
   {v2::k_vjp2<D, H1, H2, N, true, false>, v2::k_vjp2<D, H1, H2, N, true, true>}}
#define CNF_V2(D, H1, H2) {D, H1, H2, {CNF_V2N(D, H1, H2, 1), CNF_V2N(D, H1, H2, 2)}}


}  // namespace cnf
