// Fused multi-layer coupling kernel for the narrow calibration flows whose
// every conditioner Linear fits 32 floats (W[nout][nin] + b[nout]: the
// reference default D=10, hidden_size=[5,5], flows/flows.py:71, is three 5x5
// Linears per net).  Serves every final-output launch of those shapes:
// forward (+log-det), inverse, the fused calibrator eval loss and the fused
// predict pass.
//
// (Every-layer outputs, the reference's zs / xs lists, are served by k_valu:
// its LDS-staged stores are faster for the L*B*D floats.)
//
// Reference semantics restated (paths in the reference repo):
//   MLP.forward                 flows/utils.py:26-31
//   NvpCouplingLayer.forward    flows/flows.py:101-112
//       z = m*x + (1-m)*(x*exp(s) + t);  ld = sum((1-m)*s);  z = z[:,perm]; z.flip(1)
//   NvpCouplingLayer.backward   flows/flows.py:114-126  (the INVERSE)
//       z = z.flip(1); z = z[:,rev_perm]; x = m*z + (1-m)*(z-t)*exp(-s); ld = -sum((1-m)s)
//   Flow.forward / backward     flows/flows.py:17-37
//   calibrator loss terms       calibrators.py:287-291, 297-317 (CE variant:
//                               run_experiment3D.py:107)
//   predict                     calibrators.py:40-44, 330-353:
//       softmax(log(softmax(flow(x - mean x)) + 1e-7) - log_priors)
//
// Work layout.  A WAVE owns a tile of 128 consecutive rows; lane l holds rows
// 2l and 2l+1 as one packed pair per feature, so every conditioner FMA is one
// v_pk_fma_f32 for two rows with the weight as an SGPR operand:
//   * weights: each Linear's block is pulled into SGPRs by s_load_dwordx16
//     issued one Linear ahead of its use (double-buffered, 64 SGPRs); the
//     bias rides the first FMA of each neuron as the high half of its weight's
//     SGPR pair (op_sel);
//   * ReLU costs nothing: the hidden Linears are stored scaled by 2^-64
//     (cnf_prepare) so relu(a) * 2^-64 = clamp(a * 2^-64, 0, 1) is the clamp
//     bit of the neuron's last FMA; the next Linear's input columns carry the
//     2^64 back (powers of two: exact, no rounding change).  Activations past
//     2^64 (1.8e19) would saturate -- those rows overflow exp(s) anyway;
//   * the s-net's last Linear is stored pre-multiplied by log2(e), so exp(s) is
//     one v_exp_f32 and the log-det is ln2 * sum(s');
//   * input: the wave's next tile streams HBM -> LDS by LDS-DMA
//     (global_load_lds_dwordx4, no VGPRs) while the current tile computes; a
//     lane's two rows are 2*D contiguous floats, so each feature pair is one
//     ds_read2_b32 straight into a packed register pair;
//   * output: the lane writes its rows into the wave's LDS tile (the input
//     tile's rows are in registers by then, ds_write2_b32 per feature pair),
//     and the wave stores the tile lane-linear with streaming 16-B stores, each
//     instruction 1 KiB contiguous; the next tile's LDS-DMA is issued once the
//     staged rows have been read back;
//   * a persistent grid (CUs x resident blocks) walks the tiles wave by wave,
//     the waves with more tiles left at higher priority (s_setprio).
// Every variant is compile-time (mode, random_flip, every-layer stores), so
// the hot loop has no data-dependent branches and no scratch.
#include <hip/hip_runtime.h>

#include <mutex>
#include <type_traits>
#include <unordered_map>

#include "cnf_internal.h"
#include "cnf_valu_common.h"
#include "cnf_valu_io.h"
#include "cnf_sgpr_common.h"

#ifdef CNF_SGPR_TRACE
// Diagnostic build only (make trace, never shipped): per-wave s_memrealtime
// (100 MHz) marks [start, tile0 data, tile0 done, tile1 data, tile1 done,
// last tile done, end, hw id] of the last launch, read by tools/sgpr_trace.py.
__device__ unsigned long long cnf_trace[16384 * 8];
// shader-clock stamps (s_memtime) at the wave's start and end: the in-kernel
// clock is their difference over the s_memrealtime (100 MHz) difference
__device__ unsigned long long cnf_trace_clk[16384 * 2];
#define CNF_TRC(slot)                                                                   \
  do {                                                                                  \
    if (lane == 0 && gw < 16384) cnf_trace_clk[gw * 2 + (slot)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#define CNF_TR(slot)                                                                   \
  do {                                                                                 \
    if (lane == 0 && gw < 16384) cnf_trace[gw * 8 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define CNF_TR(slot) \
  do {               \
  } while (0)
#define CNF_TRC(slot) \
  do {                \
  } while (0)
#endif

namespace cnf {
namespace {

using namespace valu;

constexpr int kWaves = 4;  // waves per block

// One row pair per lane (two rows, one packed register per feature).  Two
// pairs per lane (half the scalar-load traffic per row, 4 waves per SIMD) were
// no faster for the forward pass and 7-19 % slower for the fused loss pass;
// 8- and 12-wave blocks, a second LDS tile per wave (the next tile's DMA ahead
// of the compute), 16-B stores straight from registers, 5 or 7 waves per SIMD,
// priority schedules other than tiles-remaining and in-launch sums of the loss
// records were measured and lost.
template <bool ALL, bool PERM>
constexpr int pairs_per_lane() { return 1; }
// resident waves per SIMD (the register budget): 6, or 4 for random_flip
// stacks (the permuted gathers)
template <int MODE, bool ALL, bool PERM>
constexpr int waves_per_simd() { return PERM ? 4 : 6; }

enum Mode { kFwd = 0, kInv = 1, kLoss = 2, kPredict = 3 };



// Conditioner activations of the lane's P row pairs (pair-major).
template <int D, int H1, int H2, int P>
struct Act {
  f2 c[P][D - D / 2];           // conditioning half (the masked input)
  f2 h1[P][H1 > 0 ? H1 : 1];
  f2 h2[P][H2 > 0 ? H2 : 1];
  f2 t[P][D / 2];               // t-net output, consumed by the s-net's last Linear
};

// One Linear for the lane's P pairs: neuron o = b[o] + sum_k W[o][k] x(q, k)
// from an SGPR block of rows [w_o0, b_o, w_o1 .. w_o(NIN-1)] at stride S;
// RELU: clamped last FMA.  The FMAs run input-major (k outer, neurons inner),
// so a wave issues NOUT * P independent chains back to back: a lone dependent
// v_pk_fma_f32 chain issues at half rate (tools/ubench/valu_chain.hip: 9.5
// vs 5.5 cycles per FMA for one wave, 5.3 vs 4.6 at five waves per SIMD).
// emit(o, a[P]) consumes neuron o once all are done; before() issues the
// next block's load once this block has landed.
template <int NIN, int NOUT, int S, bool RELU, int P, int NC, class X, class E, class F>
__device__ __forceinline__ void slin(const SW<NC>& w, X&& x, E&& emit, F&& before) {
  sready();
  before();
  f2 a[NOUT][P];
#pragma unroll
  for (int o = 0; o < NOUT; ++o)
#pragma unroll
    for (int q = 0; q < P; ++q) {
      if constexpr (RELU && NIN == 1) a[o][q] = fma_wb_clamp(w.pair(o * S), x(q, 0));
      else a[o][q] = fma_wb(w.pair(o * S), x(q, 0));
    }
#pragma unroll
  for (int k = 1; k < NIN; ++k)
#pragma unroll
    for (int o = 0; o < NOUT; ++o)
#pragma unroll
      for (int q = 0; q < P; ++q) {
        if (RELU && k == NIN - 1) a[o][q] = fma_ws_clamp(w, o * S + 1 + k, x(q, k), a[o][q]);
        else a[o][q] = fma_ws(w, o * S + 1 + k, x(q, k), a[o][q]);
      }
#pragma unroll
  for (int o = 0; o < NOUT; ++o) emit(o, a[o]);
}

// Float offset of Linear IDX in a layer's block when the t-net runs first
// (storage keeps the state_dict order: s-net, then t-net).
template <class S, int NETS, int IDX>
__device__ __forceinline__ constexpr int lin_at() {
  return ((NETS == 2 && IDX < S::NL) ? S::NF : 0) + S::off(IDX % S::NL);
}

// Linear IDX of a layer's sequence: the t-net's Linears, then the s-net's, so
// the s-net's last Linear applies the affine update neuron by neuron and each
// s value is consumed as it is produced (upd).  The next block (or the next
// layer's first, wn) is issued before the FMAs.  The two SGPR buffers
// alternate by the Linear's parity in the layer pair (PAR) -- never a
// `cur = nxt` copy, which would let the compiler move an in-flight s_load
// destination before its wait.
template <class S, int NETS, int P, int IDX, int PAR, bool NEXT, class AC, class U>
__device__ __forceinline__ void run_seq(AC& ac, SW<S::NC>& A, SW<S::NC>& Bf, const float* wl,
                                        const float* wn, U&& upd) {
  constexpr int NL = S::NL, N = NETS * NL;
  if constexpr (IDX < N) {
    constexpr int i = IDX % NL;
    constexpr bool tnet = IDX < NL, last = i == NL - 1;
    constexpr bool odd = ((IDX + PAR) & 1) != 0;
    SW<S::NC>& cur = odd ? Bf : A;
    SW<S::NC>& nxt = odd ? A : Bf;
    auto x = [&](int q, int k) -> f2 {
      if constexpr (i == 0) return ac.c[q][k];
      else if constexpr (i == 1) return ac.h1[q][k];
      else return ac.h2[q][k];
    };
    auto emit = [&](int o, const f2* a) {
#pragma unroll
      for (int q = 0; q < P; ++q) {
        if constexpr (!last) {
          if constexpr (i == 0) ac.h1[q][o] = a[q];
          else ac.h2[q][o] = a[q];
        } else if constexpr (tnet && NETS == 2) {
          ac.t[q][o] = a[q];
        }
      }
      if constexpr (last && (!tnet || NETS == 1)) upd(o, a);
    };
    slin<S::nin(i), S::nout(i), S::stride(i), !last, P>(cur, x, emit, [&]() {
      if constexpr (IDX + 1 < N)
        sissue(nxt, wl + lin_at<S, NETS, IDX + 1>());
      else if constexpr (NEXT)
        sissue(nxt, wn + lin_at<S, NETS, 0>());
    });
    run_seq<S, NETS, P, IDX + 1, PAR, NEXT>(ac, A, Bf, wl, wn, upd);
  }
}

// One coupling layer on the lane's P pairs v[P][D], input in orientation O
// (O: row held reversed), output in orientation !O -- the flip is a register
// renaming.  O is also the layer's position in its pair (the second layer's
// Linears start on buffer parity NETS * NL).  NEXT: prefetch the next layer's
// first block (wn) -- the pair's first layer does; the pair's last does not,
// so no SGPR buffer lives across the layer loop's back-edge (a loop-carried
// buffer makes the allocator rotate it through spill lanes).
template <int D, int H1, int H2, bool INV, bool O, int NETS, bool PERM, bool NEXT, int P>
__device__ __forceinline__ void sp_step(f2 (&v)[P][D], f2 (&ld)[P], SW<SP<D, H1, H2>::NC>& A,
                                        SW<SP<D, H1, H2>::NC>& Bf, const float* wl,
                                        const float* wn, bool perm,
                                        const int32_t* __restrict__ q) {
  using S = SP<D, H1, H2>;
  constexpr int DT = S::DT, DC = S::DC;
  constexpr bool OC = INV ? !O : O;
  if constexpr (INV && PERM) {
    if (perm) {  // flows/flows.py:115-117
#pragma unroll
      for (int p = 0; p < P; ++p) permute<D, O>(v[p], q);
    }
  }
  Act<D, H1, H2, P> ac;
#pragma unroll
  for (int p = 0; p < P; ++p)
#pragma unroll
    for (int k = 0; k < DC; ++k) ac.c[p][k] = v[p][R<D, OC>(DT + k)];
  // z_j = x_j * exp(s_j) + t_j (inverse: (x_j - t_j) * exp(-s_j)), s_j = log2(e) s
  // as stored, so exp(s) = 2^s_j and ld accumulates s_j (scaled by ln2 once)
  auto upd = [&](int j, const f2* a) {
#pragma unroll
    for (int p = 0; p < P; ++p) {
      f2& x = v[p][R<D, OC>(j)];
      if constexpr (NETS == 1) {  // scale=False: s = 0, exp(0) = 1, log-det += 0
        x = INV ? x - a[p] : x + a[p];
      } else if constexpr (!INV) {
        x = fmaV(x, exp2T(a[p]), ac.t[p][j]);
        ld[p] += a[p];
      } else {
        x = (x - ac.t[p][j]) * exp2T(-a[p]);
        ld[p] -= a[p];
      }
    }
  };
  run_seq<S, NETS, P, 0, O ? (NETS * S::NL) & 1 : 0, NEXT>(ac, A, Bf, wl, wn, upd);
  if constexpr (!INV && PERM) {
    if (perm) {  // flows/flows.py:110-112
#pragma unroll
      for (int p = 0; p < P; ++p) permute<D, O>(v[p], q);
    }
  }
}

// ---------------------------------------------------------------------------
// tile I/O: a lane's 2P rows (pairs p = rows 2P*l + 2p, +1) are the 2*P*D
// contiguous floats at row 2P*l of the wave's tile
// ---------------------------------------------------------------------------
// max over a row of the pair (q = 0 / 1) by v_max3_f32 (max is exact in any
// order; the fmaxf chain also canonicalised NaNs: 14 instead of 10 VALU per
// pair at D=10)
__device__ __forceinline__ float max3f(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float max2f(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
template <int D>
__device__ __forceinline__ f2 pair_max(const f2* v) {
  f2 m;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    float r = v[0][q];
    int j = 1;
#pragma unroll
    for (; j + 1 < D; j += 2) r = max3f(r, v[j][q], v[j + 1][q]);
    if (j < D) r = max2f(r, v[j][q]);
    m[q] = r;
  }
  return m;
}

// Loss terms of one pair's rows (logical order):
// CAL: loss = -(log(softmax(z)[y] + 1e-7) + ld)    calibrators.py:288-291
// CE:  loss = -log_softmax(z)[y] - det * ld         run_experiment3D.py:107
// z[y]: GATHER 1 reads it from the staged output tile (the lane's two rows at
// tile[0..D) and tile[D..2D): one ds_read_b32 per row instead of a
// ~30-instruction select tree); GATHER 0 selects from the registers (ragged
// tile).
template <int D, int GATHER>
__device__ __forceinline__ void pair_loss(const f2* v, f2 ld, uint32_t lab2, int rows, int kind,
                                          float det, float& t0, float& t1, float& t2,
                                          const float* tile) {
  const uint32_t b0 = lab2 & 0xffu, b1 = (lab2 >> 8) & 0xffu;
  const bool ok[2] = {b0 != 0xffu, b1 != 0xffu};
  constexpr float kL2E = 1.4426950408889634f, kLN2 = 0.6931471805599453f;
  float zy[2];
  if constexpr (GATHER == 1) {  // issued first: the LDS reads overlap the max / sum-exp below
    zy[0] = tile[ok[0] ? (int)b0 : 0];
    zy[1] = tile[D + (ok[1] ? (int)b1 : 0)];
  }
  const f2 m = pair_max<D>(v);
  const f2 nm = m * splat(-kL2E, f2{});
  f2 se = exp2T(fmaT(kL2E, v[0], nm));
#pragma unroll
  for (int j = 1; j < D; ++j) se += exp2T(fmaT(kL2E, v[j], nm));
  if constexpr (GATHER == 0) {
    uint32_t za[D], zb[D];
#pragma unroll
    for (int j = 0; j < D; ++j) {
      za[j] = __float_as_uint(v[j].x);
      zb[j] = __float_as_uint(v[j].y);
    }
    zy[0] = __uint_as_float(sel_tree<D>(za, ok[0] ? (int)b0 : 0, 0));
    zy[1] = __uint_as_float(sel_tree<D>(zb, ok[1] ? (int)b1 : 0, 0));
  }
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    if (q >= rows) continue;
    const float lpy = zy[q] - (m[q] + __builtin_amdgcn_logf(se[q]) * kLN2);
    const float l = ld[q];
    float ce, loss;
    if (kind == CNF_LOSS_CAL) {
      ce = -__builtin_amdgcn_logf(__builtin_amdgcn_exp2f(lpy * kL2E) + 1e-7f) * kLN2;
      loss = ce - l;
    } else {
      ce = -lpy;
      loss = ce - det * l;
    }
    if (!ok[q]) ce = loss = __builtin_nanf("");
    t0 += loss;
    t1 += ce;
    t2 += l;
  }
}

// x - mean(x) per row (the calibrator centres logits before the flow,
// calibrators.py:17,42)
// (O: the row is held reversed; the sum runs in logical order either way)
template <int D, bool O>
__device__ __forceinline__ void centre(f2* v) {
  f2 s = v[R<D, O>(0)];
#pragma unroll
  for (int j = 1; j < D; ++j) s += v[R<D, O>(j)];
  const f2 mu = s * splat(1.f / D, f2{});
#pragma unroll
  for (int j = 0; j < D; ++j) v[j] -= mu;
}

// softmax(log(softmax(z) + 1e-7) - log_priors) per row, in place
// (predict_post + Calibrator.predict, calibrators.py:40-44, 350-352)
template <int D>
__device__ __forceinline__ void pair_predict(f2* v, const float* __restrict__ lp) {
  constexpr float kL2E = 1.4426950408889634f, kLN2 = 0.6931471805599453f;
  const f2 m = pair_max<D>(v);
  const f2 nm = m * splat(-kL2E, f2{});
  f2 e[D], se = splat(0.f, f2{});
#pragma unroll
  for (int j = 0; j < D; ++j) {
    e[j] = exp2T(fmaT(kL2E, v[j], nm));
    se += e[j];
  }
  const f2 inv = f2{1.f / se.x, 1.f / se.y};
  f2 a[D];
#pragma unroll
  for (int j = 0; j < D; ++j) {
    const f2 p = e[j] * inv + splat(1e-7f, f2{});
    a[j] = f2{__builtin_amdgcn_logf(p.x), __builtin_amdgcn_logf(p.y)} * splat(kLN2, f2{}) -
           splat(lp[j], f2{});
  }
  const f2 m2 = pair_max<D>(a);
  const f2 nm2 = m2 * splat(-kL2E, f2{});
  f2 s2 = splat(0.f, f2{});
#pragma unroll
  for (int j = 0; j < D; ++j) {
    a[j] = exp2T(fmaT(kL2E, a[j], nm2));
    s2 += a[j];
  }
  const f2 inv2 = f2{1.f / s2.x, 1.f / s2.y};
#pragma unroll
  for (int j = 0; j < D; ++j) v[j] = a[j] * inv2;
}

// Launch arguments besides the read-only tables, which travel as separate
// __restrict__ kernel parameters: a pointer the compiler cannot prove
// unaliased by the kernel's stores is read with vector loads, not s_load.
// (the input rows and the batch size are the kernel's leading arguments, so
// that kernarg preloading puts them in SGPRs before the wave starts: see k_sgpr)
struct KArgs {
  float* out;             // final z / x / probabilities (nullable except predict)
  float* ld;              // per-row log-det (nullable)
  float* all;             // [L][B][D] every-layer outputs (ALL variants)
  const int64_t* y;       // labels (loss)
  float* part;            // per-block loss partials, 4 floats each (loss)
  // three unused words: they keep the argument block of the measured build
  // (the scalar loads of L / kind / det at these offsets; without them the
  // compiler schedules every variant differently)
  const void *reserved0, *reserved1, *reserved2;
  int L, kind;
  float det;
};

// The kernel.  MODE: kFwd / kInv (+ log-det), kLoss (forward + loss terms),
// kPredict (centre + forward + calibrated probabilities).  ALL: also store
// every layer's output.  PERM: some layer has a random_flip permutation.
// A lane carries P row pairs (2P rows), a wave tile 128*P rows.
template <int D, int H1, int H2, int NETS, int MODE, bool ALL, bool PERM>
//
// Argument order: the first three (rows in, batch size, weight region) are
// what a wave needs to issue its first tile's LDS-DMA and weight loads; the
// Makefile builds this file with kernarg preloading of them
// (-amdgpu-kernarg-preload-count), so they arrive in SGPRs with the wave
// instead of through dependent s_loads of the argument block.
__global__ __launch_bounds__(kWaves * 64, (waves_per_simd<MODE, ALL, PERM>())) void k_sgpr(
    const float* __restrict__ in,       // rows [B][D]
    int64_t B,
    const float* __restrict__ W,        // packed-SGPR weight region
    const int32_t* __restrict__ qtab,   // per-layer gather tables (forward or inverse)
    const int32_t* __restrict__ lflag,  // per-layer flags
    const float* __restrict__ lpri,     // log priors [D] (predict)
    KArgs a) {
  using S = SP<D, H1, H2>;
  constexpr int P = pairs_per_lane<ALL, PERM>();
  constexpr bool INV = MODE == kInv;
  constexpr int LF = NETS * S::NF;  // floats per layer
  constexpr int TR = 128 * P;       // rows per wave tile
  constexpr int TF = TR * D;        // floats per wave tile
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float* sm = smem + wv * TF;
  const int L = a.L;
  const int nfull = (int)(B / TR), ntiles = (int)((B + TR - 1) / TR);
  const int gw = blockIdx.x * kWaves + wv, nw = gridDim.x * kWaves;
  int left = gw < ntiles ? (ntiles - 1 - gw) / nw + 1 : 0;  // tiles this wave owns
  auto layer_of = [&](int i) { return INV ? L - 1 - i : i; };
  auto align_of = [](const void* q) {
    const int m = (int)(reinterpret_cast<uintptr_t>(q) & 15);
    return m == 0 ? 16 : ((m & 7) == 0 ? 8 : 4);
  };
  // (no longer read: kept because this early look at a.out shapes the
  // prologue's scalar-load schedule -- without it every variant compiles to a
  // different instruction stream than the measured build)
  [[maybe_unused]] const int al = a.out ? align_of(a.out) : 16;
  const int al_ld = a.ld ? align_of(a.ld) : 16;
  const bool y16 = MODE == kLoss && (reinterpret_cast<uintptr_t>(a.y) & 15) == 0;
  float lp[MODE == kPredict ? D : 1];
  if constexpr (MODE == kPredict) {
#pragma unroll
    for (int j = 0; j < D; ++j) lp[j] = lpri[j];
  }
  float lt0 = 0.f, lt1 = 0.f, lt2 = 0.f;

  // One tile's compute: rows in v -> outputs in v (logical order), log-det in
  // ld; every-layer stores on the way (rows valid: nr).  An odd stack's lone
  // layer runs FIRST, on a row read reversed (orientation 1: the tile loads
  // below write v[D-1-k] for feature k), so every stack leaves the layer-pair
  // loop in logical order: no unflip, and no register shuffle where the odd
  // and even paths meet (16 v_mov_b64 per tile when the lone layer ran last).
  const bool odd = (L & 1) != 0;
  auto compute = [&](f2 (&v)[P][D], f2 (&ld)[P], int64_t row0, int nr) {
#pragma unroll
    for (int p = 0; p < P; ++p) {
      if constexpr (MODE == kPredict) {
        if (odd) centre<D, true>(v[p]);
        else centre<D, false>(v[p]);
      }
      ld[p] = splat(0.f, f2{});
    }
    auto st_all = [&](int i, auto O_) {
      if constexpr (ALL) {
        constexpr bool O = decltype(O_)::value;
        f2 o[P][D];
#pragma unroll
        for (int p = 0; p < P; ++p)
#pragma unroll
          for (int j = 0; j < D; ++j) o[p][j] = v[p][R<D, O>(j)];
        store_rows<D, P>(a.all + ((int64_t)i * B + row0 + 2 * P * lane) * D, o, nr, 16);
      }
    };
    int i = 0;
    if (odd) {  // orientation 1 in, 0 out
      const int la = layer_of(0);
      const bool pa = PERM && (lflag[la] & kFlagPerm);
      const float* wa = W + (int64_t)la * LF;
      SW<S::NC> cur, alt;
      // a layer entered in orientation 1 starts on buffer parity NETS * NL
      // (sp_step's O): its first block goes to that buffer
      if constexpr (((NETS * S::NL) & 1) != 0) sissue(alt, wa + lin_at<S, NETS, 0>());
      else sissue(cur, wa + lin_at<S, NETS, 0>());
      sp_step<D, H1, H2, INV, true, NETS, PERM, false, P>(v, ld, cur, alt, wa, nullptr, pa,
                                                          qtab + la * D);
      st_all(0, std::false_type{});
      i = 1;
    }
    for (; i + 1 < L; i += 2) {
      const int la = layer_of(i), lb = layer_of(i + 1);
      const bool pa = PERM && (lflag[la] & kFlagPerm);
      const bool pb = PERM && (lflag[lb] & kFlagPerm);
      const float* wa = W + (int64_t)la * LF;
      const float* wb = W + (int64_t)lb * LF;
      SW<S::NC> cur, alt;
      sissue(cur, wa + lin_at<S, NETS, 0>());
      sp_step<D, H1, H2, INV, false, NETS, PERM, true, P>(v, ld, cur, alt, wa, wb, pa,
                                                          qtab + la * D);
      st_all(i, std::true_type{});
      sp_step<D, H1, H2, INV, true, NETS, PERM, false, P>(v, ld, cur, alt, wb, nullptr, pb,
                                                          qtab + lb * D);
      st_all(i + 1, std::false_type{});
    }
#pragma unroll
    for (int p = 0; p < P; ++p) {
      if constexpr (NETS == 2) ld[p] = ld[p] * splat(0.69314718055994531f, f2{});  // ln2 sum(s')
      if constexpr (MODE == kPredict) pair_predict<D>(v[p], lp);
    }
  };
  // tile: the lane's staged output rows in LDS (full tiles), or nullptr
  auto loss = [&](const f2 (&v)[P][D], const f2 (&ld)[P], uint32_t lab, int nr,
                  const float* tile, auto gather) {
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const int r = nr - 2 * p;
      constexpr int G = decltype(gather)::value;
      pair_loss<D, G>(v[p], ld[p], lab >> (16 * p), r < 0 ? 0 : (r > 2 ? 2 : r), a.kind, a.det,
                      lt0, lt1, lt2, tile + 2 * D * p);
    }
  };

  // -------- full tiles: LDS-DMA in, staged lane-linear stores out --------
  CNF_TR(0);
  CNF_TRC(0);
#ifdef CNF_SGPR_TRACE
  if (lane == 0 && gw < 16384)
    cnf_trace[gw * 8 + 7] = ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |
                            __builtin_amdgcn_s_getreg((31 << 11) | 4);  // XCC_ID, HW_ID
  int ntr = 0;
#endif
  int t = gw;
  if (t < nfull) wave_dma<D, TR>(sm, in + (int64_t)t * TF, lane);
  // the wave with more tiles left goes first (VALU issue is arbitrated by
  // priority, then age): waves of one SIMD may own unequal tile counts (2^23
  // rows: 64 tiles on 6 waves; grid_for removes that only for short batches)
  auto set_prio = [&]() {
    --left;  // tiles after this one
    if (left >= 3) __builtin_amdgcn_s_setprio(3);
    else if (left == 2) __builtin_amdgcn_s_setprio(2);
    else if (left == 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
  };
  for (; t < nfull; t += nw) {
    set_prio();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA has landed
    f2 v[P][D];
    if constexpr (P == 1) {  // rows are in registers (reversed for an odd stack)
      if (odd) read_pairs_wait<D, true>(sm, lane, v);
      else read_pairs_wait<D, false>(sm, lane, v);
    } else {
      if (odd) read_pairs<D, P, true>(sm, lane, v);
      else read_pairs<D, P, false>(sm, lane, v);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
#ifdef CNF_SGPR_TRACE
    if (ntr < 2) CNF_TR(1 + 2 * ntr);
#endif
    const int64_t row0 = (int64_t)t * TR;
    uint32_t lab = 0;
    if constexpr (MODE == kLoss) lab = load_labels<D, P>(a.y + row0 + 2 * P * lane, 2 * P, y16);
    f2 ld[P];
    compute(v, ld, row0, 2 * P);
    if constexpr (MODE == kLoss) {
      // staged first: the loss reads z[y] back from the tile
      stage_pairs<D, P>(sm, lane, v);
      loss(v, ld, lab, 2 * P, sm + 2 * P * D * lane, std::integral_constant<int, 1>{});
    }
#ifdef CNF_SGPR_TRACE
    if (ntr < 2) CNF_TR(2 + 2 * ntr);
    CNF_TR(5);
    ++ntr;
#endif
    // stage in the input tile (its rows are in registers), store lane-linear,
    // then let the next tile's DMA in once the staged reads have completed
    if (a.out) {
      if (MODE != kLoss) stage_pairs<D, P>(sm, lane, v);
      store_tile<TF>(a.out + row0 * D, sm, lane);
    }
    if (a.ld) store_lds<P>(a.ld + row0 + 2 * P * lane, ld, 2 * P, al_ld);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (t + nw < nfull) wave_dma<D, TR>(sm, in + (int64_t)(t + nw) * TF, lane);
  }
  // -------- the ragged last tile (B % TR rows): plain loads, masked stores --------
  if (t == nfull && nfull < ntiles) {
    const int64_t row0 = (int64_t)t * TR;
    const int64_t r = row0 + 2 * P * lane;
    const int64_t left_rows = B - r;
    const int nr = left_rows <= 0 ? 0 : (left_rows >= 2 * P ? 2 * P : (int)left_rows);
    f2 v[P][D];
    auto load_rows = [&](auto O_) {
      constexpr bool O = decltype(O_)::value;
#pragma unroll
      for (int p = 0; p < P; ++p)
#pragma unroll
        for (int k = 0; k < D; ++k) {
          v[p][R<D, O>(k)].x = 2 * p < nr ? in[(r + 2 * p) * D + k] : 0.f;
          v[p][R<D, O>(k)].y = 2 * p + 1 < nr ? in[(r + 2 * p + 1) * D + k] : 0.f;
        }
    };
    if (odd) load_rows(std::true_type{});
    else load_rows(std::false_type{});
    uint32_t lab = 0;
    if constexpr (MODE == kLoss) lab = load_labels<D, P>(a.y + r, nr, false);
    f2 ld[P];
    compute(v, ld, row0, nr);
    if constexpr (MODE == kLoss) loss(v, ld, lab, nr, sm, std::integral_constant<int, 0>{});
    if (a.out) store_rows<D, P>(a.out + r * D, v, nr, 4);
    if (a.ld) store_lds<P>(a.ld + r, ld, nr, 4);
  }
  CNF_TRC(1);
  CNF_TR(6);
  if constexpr (MODE == kLoss) block_sum3<kWaves * 64>(lt0, lt1, lt2, smem, a.part);
}

using KFn = void (*)(const float*, int64_t, const float*, const int32_t*, const int32_t*,
                     const float*, KArgs);

// one instantiation and the rows of its wave tile
struct KV {
  KFn fn;
  int tr;
};

// variants without permutation: fwd, inv, loss, predict; with a random_flip
// permutation: fwd, inv, predict.  The every-layer-output form (ALL) is not
// instantiated: those launches go to k_valu, whose LDS-staged stores write
// the L*B*D floats faster (cnf_valu.hip valu_run); ALL stays as a template
// switch for A/B builds.
enum Var { vFwd, vInv, vLoss, vPredict, kNVar };

struct SEntry {
  int D, H1, H2;
  KV fn[2][kNVar];  // [nets - 1][variant]
  KV pfn[2][3];     // [nets - 1][fwd, inv, predict] with permutation
};

#define CNF_K(D, H1, H2, N, M, A, P) \
  {k_sgpr<D, H1, H2, N, M, A, P>, 128 * pairs_per_lane<A, P>()}
#define CNF_SV(D, H1, H2, N)                                                                  \
  {CNF_K(D, H1, H2, N, kFwd, false, false), CNF_K(D, H1, H2, N, kInv, false, false),           \
   CNF_K(D, H1, H2, N, kLoss, false, false), CNF_K(D, H1, H2, N, kPredict, false, false)}
#define CNF_SP(D, H1, H2, N)                                                                  \
  {CNF_K(D, H1, H2, N, kFwd, false, true), CNF_K(D, H1, H2, N, kInv, false, true),             \
   CNF_K(D, H1, H2, N, kPredict, false, true)}
#define CNF_SGPR(D, H1, H2) \
  {D, H1, H2, {CNF_SV(D, H1, H2, 1), CNF_SV(D, H1, H2, 2)}, {CNF_SP(D, H1, H2, 1), CNF_SP(D, H1, H2, 2)}}

// every shape of the VALU table whose Linears fit the 32-float buffer
const SEntry kSTable[] = {
#ifdef CNF_SGPR_DEV  // development builds: the headline shape only
    CNF_SGPR(10, 5, 5),
#else
    CNF_SGPR(2, 5, 5), CNF_SGPR(3, 5, 5), CNF_SGPR(4, 5, 5), CNF_SGPR(5, 5, 5),
    CNF_SGPR(6, 5, 5), CNF_SGPR(8, 5, 5), CNF_SGPR(10, 5, 5),
    CNF_SGPR(3, 3, 3), CNF_SGPR(8, 3, 3), CNF_SGPR(10, 3, 3),
    CNF_SGPR(3, 3, 0), CNF_SGPR(3, 0, 0), CNF_SGPR(10, 0, 0),
    CNF_SGPR(10, 5, 0), CNF_SGPR(3, 5, 0),
#endif
};

const SEntry* find(const Shape& s) {
  const int h1 = s.n_lin >= 2 ? s.units[1] : 0, h2 = s.n_lin >= 3 ? s.units[2] : 0;
  for (const SEntry& e : kSTable)
    if (e.D == s.D && e.H1 == h1 && e.H2 == h2) return &e;
  return nullptr;
}

size_t lds_bytes(const Shape& s, const KV& k) {
  return (size_t)kWaves * k.tr * s.D * 4;
}

int resident_blocks(const KV& k, size_t lds) {
  static std::mutex mu;
  static std::unordered_map<const void*, int> cache;
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find((const void*)k.fn);
  if (it != cache.end()) return it->second;
  int n = 0, dev = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k.fn, kWaves * 64, lds) != hipSuccess ||
      n < 1)
    n = 1;
  // at most kGridWps blocks per CU even where the occupancy query
  // allows more: at 7 per CU (forward, 71 VGPRs) the last ~10 % of a 2^20-row
  // grid was not resident at launch and started ~18 us late (tools/sgpr_trace.py).
  // 6 (with the 6-wave register budget, 80 VGPRs, no scratch) measured 0.6-0.8 us
  // faster per 2^20-row loss / forward call than 5 (round 4, two interleaved
  // A/B passes); 7 spills the loss build
  constexpr int kGridWps = 6;
  if (n > kGridWps * 4 / kWaves) n = kGridWps * 4 / kWaves;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus < 1)
    cus = 256;
  cache[(const void*)k.fn] = n * cus;
  return n * cus;
}

const KV* pick(const SEntry* e, const Shape& s, int mode, bool all) {
  const int n = s.scale ? 1 : 0;
  if (all) return nullptr;  // k_valu serves every-layer outputs
  if (s.any_perm) {
    if (mode == kLoss) return nullptr;  // k_valu handles the permuted fused eval
    return &e->pfn[n][mode == kInv ? 1 : (mode == kPredict ? 2 : 0)];
  }
  return &e->fn[n][mode];
}

// persistent grid: every wave of a resident block walks tiles
int64_t grid_for(const KV& k, const Shape& s, int64_t B) {
  const int64_t ntiles = (B + k.tr - 1) / k.tr;
  const int64_t want = (ntiles + kWaves - 1) / kWaves;
  int64_t cap = resident_blocks(k, lds_bytes(s, k));
  // A short batch whose tiles fall evenly on the SIMDs but not on their
  // resident waves ends in a tail at low occupancy (2^20 rows: 8 tiles per
  // SIMD on 6 waves run as 6, then 2 on 2 waves).  There, the largest count
  // of waves per SIMD (at least 4) that divides the tiles runs them in full
  // rounds instead; longer batches keep every resident wave (their tail is
  // a small share, and more waves hide more latency).  2^20 rows: 29.36 vs
  // 30.31 us per loss call, 24.54 vs 25.05 us forward; 2^21 -0.5 / -1.5 %
  // (profiles/r06_ab_even_grid.jsonl).
  static const int cus = []() {
    int dev = 0, c = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        c < 1)
      c = 256;
    return c;
  }();
  const int64_t simds = (int64_t)cus * 4, wmax = cap / cus;
  if (ntiles % simds == 0) {
    const int64_t T = ntiles / simds;
    if (T <= 24 && T % wmax != 0)
      for (int64_t w = wmax - 1; w >= 4; --w)
        if (T % w == 0) {
          cap = w * cus;
          break;
        }
  }
  return want < cap ? want : cap;
}

bool io_ok(const void* p, int64_t align) {
  return p == nullptr || (reinterpret_cast<uintptr_t>(p) % align) == 0;
}

}  // namespace

// Shapes this kernel serves: shift on (NICE keeps s = 0), non-strict, every
// Linear fits 32 floats, and the row batch in HBM is 16-B aligned (the LDS-DMA
// reads whole 16-B words; misaligned views stay on k_valu).
bool sgpr_enabled(const Shape& s) {
  return s.sp_ok && !s.strict && s.shift && !s.alt_mask && !s.s_tanh && find(s) &&
         !(s.options & CNF_OPT_NO_SGPR);
}

int64_t sgpr_blocks(const Shape& s, int64_t B) {
  const SEntry* e = find(s);
  const KV* k = e ? pick(e, s, kLoss, false) : nullptr;
  return k ? grid_for(*k, s, B) : 0;
}

int sgpr_run(const Shape& s, const void* prepared, const float* in, float* out, float* ld,
             float* all, int64_t B, bool inverse, hipStream_t st, const int64_t* y,
             float* loss_ws, int kind, float det, float* loss_terms, const float* log_priors) {
  const SEntry* e = find(s);
  if (!e || !sgpr_enabled(s)) return CNF_ERR_UNSUPPORTED;
  if (B == 0) return CNF_OK;
  if (B / 128 > 0x7fffffffLL) return CNF_ERR_UNSUPPORTED;
  // staged tile stores write whole 16-B words: a misaligned output view stays on k_valu
  if (!io_ok(in, 16) || !io_ok(out, 16) || !io_ok(all, 16) || !io_ok(ld, 4))
    return CNF_ERR_UNSUPPORTED;
  const int mode = log_priors ? kPredict : (loss_ws ? kLoss : (inverse ? kInv : kFwd));
  const KV* k = pick(e, s, mode, all != nullptr);
  if (!k) return CNF_ERR_UNSUPPORTED;
  const char* base = static_cast<const char*>(prepared);
  const int32_t* fwd_q = reinterpret_cast<const int32_t*>(base);
  const int32_t* inv_q = fwd_q + s.L * s.D;
  const int32_t* flags = inv_q + s.L * s.D;
  const float* W = reinterpret_cast<const float*>(base + idx_bytes(s)) + s.sp_region;
  KArgs a{};
  a.out = out;
  a.ld = ld;
  a.all = all;
  a.y = y;
  a.part = loss_ws ? loss_ws + 4 : nullptr;
  a.L = s.L;
  a.kind = kind;
  a.det = det;
  const int64_t nblk = grid_for(*k, s, B);
  hipLaunchKernelGGL(k->fn, dim3((unsigned)nblk), dim3(kWaves * 64), lds_bytes(s, *k), st, in, B,
                     W, inverse ? inv_q : fwd_q, flags, log_priors, a);
  // the block-order sum of the loss records: a one-block follow-up launch
  // (in-launch sums measured slower: cnf_valu_io.h reduce_rows4_block)
  if (mode == kLoss) reduce_partials(loss_ws + 4, (int)nblk, 4, 0, nullptr, loss_terms, st);
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    set_hip_error(err);
    return CNF_ERR_HIP;
  }
  return CNF_OK;
}

}  // namespace cnf

#ifdef CNF_SGPR_TRACE
extern "C" int cnf_diag_trace_clk(unsigned long long* host, int n) {
  if (n > 16384 * 2) n = 16384 * 2;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(cnf_trace_clk), (size_t)n * 8, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? n : -1;
}
extern "C" int cnf_diag_trace(unsigned long long* host, int n) {
  if (n > 16384 * 8) n = 16384 * 8;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(cnf_trace), (size_t)n * 8, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? n : -1;
}
#endif
