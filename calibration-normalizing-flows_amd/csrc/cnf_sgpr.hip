// Fused multi-layer coupling kernel, pipelined-scalar-weight form, for the
// narrow calibration flows whose every conditioner Linear fits 32 floats
// (W[nout][nin] + b[nout]: the reference default D=10, hidden_size=[5,5],
// flows/flows.py:71, is three 5x5 Linears per net).
//
// Same math and tile/row layout as k_valu (cnf_valu.hip header comment,
// flows/flows.py:101-126), different weight path: every Linear's block is
// pulled into SGPRs by two s_load_dwordx16 issued one Linear AHEAD of its use
// (double-buffered, 64 SGPRs), so
//   * each FMA takes its weight as an SGPR operand (op_sel picks the half),
//     with no VGPR copies of weights and no LDS broadcast traffic;
//   * the scalar-cache round trip of a Linear overlaps the previous Linear's
//     FMAs instead of stalling the wave once per output neuron.
// The s-net's last Linear is stored pre-multiplied by log2(e) (cnf_prepare), so
// exp(s) is one v_exp_f32 and the log-det is ln2 * sum(s') once per row.
// Non-strict only (strict_nan keeps k_valu); shift must be on (NICE: s = 0).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <mutex>
#include <unordered_map>

#include "cnf_internal.h"
#include "cnf_valu_common.h"
#include "cnf_valu_io.h"

#ifndef CNF_SGPR_WPE
#define CNF_SGPR_WPE 5
#endif

#ifdef CNF_TIMELINE
// Diagnostic build only (make timeline): per-block wall-clock marks of the
// persistent kernel, s_memrealtime (100 MHz): [start, first tile ready, end, hw id]
__device__ unsigned long long cnf_tl[4096 * 4];
#endif

namespace cnf {
namespace {

using namespace valu;

#ifdef CNF_TIMELINE
__device__ __forceinline__ void tl_mark(int slot) {
  if (threadIdx.x == 0 && blockIdx.x < 4096) {
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    cnf_tl[blockIdx.x * 4 + slot] = t;
    if (slot == 0)
      cnf_tl[blockIdx.x * 4 + 3] =
          ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |
          __builtin_amdgcn_s_getreg((31 << 11) | 4);  // XCC_ID, HW_ID
  }
}
#define CNF_TL(slot) tl_mark(slot)
#else
#define CNF_TL(slot)
#endif

// Compile-time SP layout of one net (must match derive_shape's sp_lin_off).
template <int D, int H1, int H2>
struct SP {
  static constexpr int DT = D / 2, DC = D - D / 2;
  static constexpr int NL = H1 == 0 ? 1 : (H2 == 0 ? 2 : 3);
  static constexpr int nin(int i) { return i == 0 ? DC : (i == 1 ? H1 : H2); }
  static constexpr int nout(int i) { return i == NL - 1 ? DT : (i == 0 ? H1 : H2); }
  // per output row: [w_o0, b_o, w_o1 .. w_o(nin-1)], row stride even so that
  // (w_o0, b_o) is one aligned SGPR pair
  static constexpr int stride(int i) { return (nin(i) + 2) & ~1; }
  static constexpr int fl(int i) { return pad16(nout(i) * stride(i)); }
  static constexpr int off(int i) { return i == 0 ? 0 : off(i - 1) + fl(i - 1); }
  static constexpr int NF = off(NL);
  static constexpr int mx(int i) { return i == NL ? 0 : (fl(i) > mx(i + 1) ? fl(i) : mx(i + 1)); }
  static constexpr int NC = mx(0) / 16;  // 64-B chunks per buffer
  static_assert(NC >= 1 && NC <= 2, "Linear block exceeds the 32-float SGPR buffer");
};

template <int NC>
struct SW {
  v16f c[NC];
  __device__ __forceinline__ float operator[](int i) const { return c[i >> 4][i & 15]; }
  __device__ __forceinline__ f2 pair(int i) const {  // i even
    return f2{c[i >> 4][i & 15], c[i >> 4][(i & 15) + 1]};
  }
};

// w0 * x + b with (w0, b) ONE SGPR pair: op_sel broadcasts the low half as the
// multiplier and the high half as the addend, so the bias costs no VALU move
// (a pair read twice is one constant-bus operand).
__device__ __forceinline__ f2 fma_wb(f2 wb, f2 x) {
  f2 a;
  asm("v_pk_fma_f32 %0, %1, %2, %1 op_sel:[0,0,1] op_sel_hi:[0,1,1]" : "=v"(a) : "s"(wb), "v"(x));
  return a;
}

// Issue the loads of one Linear block: plain (compiler-visible) scalar loads,
// so the compiler's own s_waitcnt insertion guards every read of the
// destination SGPRs -- including any copy or spill the register allocator
// adds -- and a sched_barrier keeps the load from sinking toward its use:
// ALU work may cross it, memory operations may not, so the block's
// s_load_dwordx16 pair issues one Linear ahead of its first FMA.
// (An earlier form issued the s_load from inline asm and waited in a second
// asm statement; the allocator was then free to copy the in-flight
// destination registers between the two -- seen as s_mov_b64 of a pending
// s_load_dwordx16 destination -- i.e. to read weights before they landed.)
template <int NC>
__device__ __forceinline__ void sissue(SW<NC>& r, const float* p) {
  const v16f* q = reinterpret_cast<const v16f*>(__builtin_assume_aligned(p, 64));
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < NC; ++i) r.c[i] = q[i];
  __builtin_amdgcn_sched_barrier(0);
}
// End of the Linear that overlaps the load: nothing crosses, so the next
// Linear's FMAs (the loaded block's consumers) cannot be hoisted up to the load.
template <int NC>
__device__ __forceinline__ void swait(SW<NC>&) {
  __builtin_amdgcn_sched_barrier(0);
}

// y[o] = b[o] + sum_k W[o][k] x[k] from an SGPR block of rows
// [w_o0, b_o, w_o1 .. w_o(NIN-1)] at stride S (even)
// after(): issued once the first output neuron is done (the next block's load:
// the compiler's wait for THIS block then precedes it, so an SMEM lgkmcnt(0)
// never has to cover the load just issued).
template <int NIN, int NOUT, int S, bool RELU, int NC, class T, class F>
__device__ __forceinline__ void slin(const SW<NC>& w, const T* x, T* y, F&& after) {
  static_assert(sizeof(T) == 8, "pipelined-scalar kernel packs two rows per lane");
#pragma unroll
  for (int o = 0; o < NOUT; ++o) {
    T a = fma_wb(w.pair(o * S), x[0]);
#pragma unroll
    for (int k = 1; k < NIN; ++k) a = fmaT(w[o * S + 1 + k], x[k], a);
    y[o] = RELU ? relu<false>(a) : a;
    if (o == 0) after();
  }
}

// Linear IDX of the layer's sequence (net-major: s-net Linears, then t-net);
// the next block (or the next layer's first, wn) is issued before computing.
// The two SGPR buffers alternate by the Linear's parity in the layer pair
// (PAR: parity of the layer's first Linear) -- never a `cur = nxt` copy: a
// copy gives the compiler a reason to move the in-flight destination of an
// s_load into other registers before the s_waitcnt (seen: s_mov_b64 of a
// pending s_load_dwordx16 destination), i.e. to read it before it lands.
template <class S, int NETS, int IDX, int PAR, class T>
__device__ __forceinline__ void run_seq(const T* c, T* h1, T* h2, T* s, T* t, SW<S::NC>& A,
                                        SW<S::NC>& Bf, const float* wl, const float* wn) {
  if constexpr (IDX < NETS * S::NL) {
    constexpr int net = IDX / S::NL, i = IDX % S::NL;
    constexpr bool odd = ((IDX + PAR) & 1) != 0;
    SW<S::NC>& cur = odd ? Bf : A;
    SW<S::NC>& nxt = odd ? A : Bf;
    constexpr bool last = i == S::NL - 1;
    const T* in = i == 0 ? c : (i == 1 ? h1 : h2);
    T* out = last ? ((NETS == 2 && net == 0) ? s : t) : (i == 0 ? h1 : h2);
    slin<S::nin(i), S::nout(i), S::stride(i), !last>(cur, in, out, [&]() {
      if constexpr (IDX + 1 < NETS * S::NL)
        sissue(nxt, wl + ((IDX + 1) / S::NL) * S::NF + S::off((IDX + 1) % S::NL));
      else
        sissue(nxt, wn);
    });
    swait(nxt);
    run_seq<S, NETS, IDX + 1, PAR>(c, h1, h2, s, t, A, Bf, wl, wn);
  }
}

// One coupling layer, input in orientation O, output in orientation !O
// (k_valu's step(), non-strict, weights from the pipelined SGPR buffer).
// O is also the layer's position in its pair (the odd tail layer is a first):
// the second layer's Linears start on buffer parity NETS * NL.
template <int D, int H1, int H2, bool INV, bool O, int NETS, class T>
__device__ __forceinline__ void sp_step(T* v, T& ld, SW<SP<D, H1, H2>::NC>& A,
                                        SW<SP<D, H1, H2>::NC>& Bf, const float* wl,
                                        const float* wn, bool perm,
                                        const int32_t* __restrict__ q) {
  using S = SP<D, H1, H2>;
  constexpr int DT = S::DT, DC = S::DC;
  constexpr bool OC = INV ? !O : O;
  if constexpr (INV) {
    if (perm) permute<D, O>(v, q);  // flows/flows.py:115-117
  }
  T c[DC];
#pragma unroll
  for (int k = 0; k < DC; ++k) c[k] = v[R<D, OC>(DT + k)];
  T h1[H1 > 0 ? H1 : 1], h2[H2 > 0 ? H2 : 1], s[DT], t[DT];
  run_seq<S, NETS, 0, O ? (NETS * S::NL) & 1 : 0>(c, h1, h2, s, t, A, Bf, wl, wn);
#pragma unroll
  for (int j = 0; j < DT; ++j) {
    T& x = v[R<D, OC>(j)];
    if constexpr (NETS == 1) {  // scale=False: s = 0, exp(0) = 1, log-det += 0
      x = INV ? x - t[j] : x + t[j];
    } else if constexpr (!INV) {  // s[j] = log2(e) * s (scaled at prepare): exp(s) = 2^s[j]
      x = fmaV(x, exp2T(s[j]), t[j]);
      ld += s[j];
    } else {
      x = (x - t[j]) * exp2T(-s[j]);
      ld -= s[j];
    }
  }
  if constexpr (!INV) {
    if (perm) permute<D, O>(v, q);  // flows/flows.py:110-112
  }
}

// Async copy of one full input tile (TF floats, 16-B aligned) into LDS: every
// wave moves 1 KiB per global_load_lds_dwordx4, lane-linear (the tile is
// contiguous in HBM and in LDS, so the image is the row-major tile itself).
template <int ROWS, int TF>
__device__ __forceinline__ void tile_prefetch(float* sm, const float* __restrict__ src) {
  static_assert(TF % 4 == 0, "tile must be whole float4s");
  constexpr int N4 = TF / 4, NI = (N4 + 63) / 64, NW = ROWS / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < (NI + NW - 1) / NW; ++i) {
    const int c = (i * NW + w) * 64;  // first float4 of this wave's 1 KiB
    if (c + lane < N4)
      __builtin_amdgcn_global_load_lds(src + (int64_t)(c + lane) * 4,
                                       (__attribute__((address_space(3))) void*)(sm + c * 4), 16,
                                       0, 0);
  }
}

// Per-wave form: wave w copies only the rows it owns (rows q*ROWS + 64w ..
// +63 of the tile, RW contiguous 64*D-float chunks) into the same place of the
// LDS image, so it waits on its own vmcnt and needs no block barrier before
// reading them or before refilling them with the next tile.
template <int D, int ROWS, int RW>
__device__ __forceinline__ void wave_prefetch(float* sm, const float* __restrict__ src) {
  constexpr int N4 = 16 * D;  // float4s per 64-row chunk
  const int lane = threadIdx.x & 63;
  // wave-uniform chunk bases in SGPRs; one lane-offset VGPR for every copy
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
  for (int q = 0; q < RW; ++q) {
    const int c0 = (q * ROWS + 64 * w) * D / 4;  // first float4 of the chunk
    const float* base = src + (int64_t)c0 * 4;
#pragma unroll
    for (int i = 0; i < (N4 + 63) / 64; ++i) {
      if (i * 64 + lane < N4)
        __builtin_amdgcn_global_load_lds(base + (i * 64 + lane) * 4,
                                         (__attribute__((address_space(3))) void*)(sm + (c0 + i * 64) * 4),
                                         16, 0, 0);
    }
  }
}

// PIPE: persistent grid (CUs x resident blocks) walking the tiles; while a
// tile computes, the next full tile streams into the LDS tile by LDS-DMA (no
// VGPRs), and outputs go straight from registers to HBM.
// PIPE: 0 one tile per block, 1 persistent + block-wide DMA, 2 persistent +
// per-wave DMA (no barriers on the tile path).
template <int D, int H1, int H2, bool INV, int NETS, int RW, int ROWS, int PIPE>
__global__ __launch_bounds__(ROWS, INV ? CNF_SGPR_WPE - 1 : CNF_SGPR_WPE) void k_sgpr(
    const float* __restrict__ W, const int32_t* __restrict__ qtab,
    const int32_t* __restrict__ lflag, const float* __restrict__ in, float* __restrict__ out,
    float* __restrict__ ld_out, float*, int64_t B, int L, int prio_mode, int,
    int any_perm, int vec_io, const int64_t* __restrict__ yl, float* __restrict__ loss_part,
    int kind, float det, unsigned* __restrict__ ticket, float* __restrict__ loss_terms) {
  using S = SP<D, H1, H2>;
  using T = typename RowT<RW>::type;
  constexpr int TR = ROWS * RW;
  constexpr int LF = NETS * S::NF;  // floats per layer
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sm = smem;
  const int tid = threadIdx.x;
  const bool vec = vec_io != 0;
  CNF_TL(0);
  const int64_t ntiles = (B + TR - 1) / TR;
  auto layer_of = [&](int i) { return INV ? L - 1 - i : i; };
  float lt0 = 0.f, lt1 = 0.f, lt2 = 0.f;

  constexpr int TF = TR * D;
  const int64_t nfull = B / TR;
  const bool dma = PIPE && vec;
  constexpr bool WDMA = PIPE == 2;
  if (dma && (int64_t)blockIdx.x < nfull) {
    if constexpr (WDMA) wave_prefetch<D, ROWS, RW>(sm, in + (int64_t)blockIdx.x * TF);
    else tile_prefetch<ROWS, TF>(sm, in + (int64_t)blockIdx.x * TF);
  }

  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    if (prio_mode) {  // longest-remaining-first: blocks with more tiles left win issue
      const int64_t rem = (ntiles - 1 - tile) / gridDim.x;  // tiles after this one
      if (rem >= 3) __builtin_amdgcn_s_setprio(3);
      else if (rem == 2) __builtin_amdgcn_s_setprio(2);
      else if (rem == 1) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
    }
    const int64_t row0 = tile * TR;
    const int nrows = (int)((B - row0) < TR ? (B - row0) : TR);
    SW<S::NC> cur, alt;
    sissue(cur, W + (int64_t)layer_of(0) * LF);  // lands while the tile loads
    int yv[RW];
    if (loss_part) load_labels<RW>(yl, row0, tid, ROWS, B, yv);
    if (dma && tile < nfull) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA has landed
      if constexpr (!WDMA) lds_barrier();               // ... and every other wave's
    } else {
      lds_barrier();
      tile_load<ROWS>(sm, in + row0 * D, nrows * D, vec);
      lds_barrier();
    }
    T v[D];
#pragma unroll
    for (int k = 0; k < D; ++k) v[k] = get_row<ROWS>(sm, tid, D, k, T{});
    if (tile == blockIdx.x) CNF_TL(1);
    if (dma) {
      const int64_t nt = tile + gridDim.x;
      if (nt < nfull) {
        if constexpr (WDMA) {
          // this wave's rows are in registers once its LDS reads return
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          wave_prefetch<D, ROWS, RW>(sm, in + nt * TF);
        } else {
          lds_barrier();  // every wave has its rows in registers
          tile_prefetch<ROWS, TF>(sm, in + nt * TF);
        }
      }
    }
    swait(cur);
    T ld = splat(0.f, T{});
    int i = 0;
    for (; i + 1 < L; i += 2) {
      const int la = layer_of(i), lb = layer_of(i + 1), lc = layer_of(i + 2 < L ? i + 2 : 0);
      const bool pa = any_perm && (lflag[la] & kFlagPerm);
      const bool pb = any_perm && (lflag[lb] & kFlagPerm);
      sp_step<D, H1, H2, INV, false, NETS>(v, ld, cur, alt, W + (int64_t)la * LF,
                                           W + (int64_t)lb * LF, pa, qtab + la * D);
      sp_step<D, H1, H2, INV, true, NETS>(v, ld, cur, alt, W + (int64_t)lb * LF,
                                          W + (int64_t)lc * LF, pb, qtab + lb * D);
    }
    const bool odd = i < L;
    if (odd) {
      const int la = layer_of(i);
      const bool pa = any_perm && (lflag[la] & kFlagPerm);
      sp_step<D, H1, H2, INV, false, NETS>(v, ld, cur, alt, W + (int64_t)la * LF,
                                           W + (int64_t)layer_of(0) * LF, pa, qtab + la * D);
    }
    if constexpr (NETS == 2) ld = ld * splat(0.69314718055994531f, T{});  // sum(s) = ln2 * sum(s')
    if (out) {
      if constexpr (PIPE) {  // the LDS tile is already the next tile's DMA target
        const bool al8 = (reinterpret_cast<uintptr_t>(out) & 7) == 0;
        if (odd) store_rows_direct<D, ROWS, true>(out + row0 * D, v, nrows, al8);
        else store_rows_direct<D, ROWS, false>(out + row0 * D, v, nrows, al8);
      } else {
        if (odd) store_rows<D, ROWS, true>(out + row0 * D, sm, v, nrows, vec);
        else store_rows<D, ROWS, false>(out + row0 * D, sm, v, nrows, vec);
      }
    }
    if (ld_out) store_ld<ROWS>(ld_out, row0, tid, nrows, ld);
    if (loss_part) {
      if (odd) tile_loss<D, true>(v, ld, yv, kind, det, lt0, lt1, lt2);
      else tile_loss<D, false>(v, ld, yv, kind, det, lt0, lt1, lt2);
    }
  }
  CNF_TL(2);
  if (loss_part) {
    if (ticket)  // persistent grid: one hand-off per block, no second launch
      block_sum3_last<ROWS>(lt0, lt1, lt2, smem, loss_part, ticket, loss_terms, gridDim.x);
    else
      block_sum3<ROWS>(lt0, lt1, lt2, smem, loss_part);
  }
}

using KFn = void (*)(const float*, const int32_t*, const int32_t*, const float*, float*, float*,
                     float*, int64_t, int, int, int, int, int, const int64_t*, float*, int, float,
                     unsigned*, float*);

constexpr int kRW = 2, kRows = 256;

struct SEntry {
  int D, H1, H2;
  KFn fn[3][2][2];  // [pipe][nets - 1][inverse]
};

#define CNF_SGPR_P(D, H1, H2, P)                                                      \
  {{k_sgpr<D, H1, H2, false, 1, kRW, kRows, P>, k_sgpr<D, H1, H2, true, 1, kRW, kRows, P>}, \
   {k_sgpr<D, H1, H2, false, 2, kRW, kRows, P>, k_sgpr<D, H1, H2, true, 2, kRW, kRows, P>}}
#define CNF_SGPR(D, H1, H2) \
  {D, H1, H2, {CNF_SGPR_P(D, H1, H2, 0), CNF_SGPR_P(D, H1, H2, 1), CNF_SGPR_P(D, H1, H2, 2)}}

// every shape of the VALU table whose Linears fit the 32-float buffer
const SEntry kSTable[] = {
    CNF_SGPR(2, 5, 5), CNF_SGPR(3, 5, 5), CNF_SGPR(4, 5, 5), CNF_SGPR(5, 5, 5),
    CNF_SGPR(6, 5, 5), CNF_SGPR(8, 5, 5), CNF_SGPR(10, 5, 5),
    CNF_SGPR(3, 3, 3), CNF_SGPR(8, 3, 3), CNF_SGPR(10, 3, 3),
    CNF_SGPR(3, 3, 0), CNF_SGPR(3, 0, 0), CNF_SGPR(10, 0, 0),
    CNF_SGPR(10, 5, 0), CNF_SGPR(3, 5, 0),
};

const SEntry* find(const Shape& s) {
  const int h1 = s.n_lin >= 2 ? s.units[1] : 0, h2 = s.n_lin >= 3 ? s.units[2] : 0;
  for (const SEntry& e : kSTable)
    if (e.D == s.D && e.H1 == h1 && e.H2 == h2) return &e;
  return nullptr;
}

}  // namespace

// all_outputs (z_all) launches stay on k_valu: the per-layer stores cost this
// kernel SGPRs it does not have.
bool sgpr_enabled(const Shape& s) {
  if (!s.sp_ok || s.strict || !s.shift || !find(s)) return false;
  const char* e = std::getenv("CNF_SGPR");  // A/B switch: CNF_SGPR=0 keeps k_valu
  return !(e && e[0] == '0');
}

// A/B switch CNF_SGPR_PIPE: 0 one tile per block, 1 block-wide DMA, 2 per-wave
// DMA (default).  A wave-granular dynamic schedule (atomic unit counters per
// XCD, per-unit loss records) was measured and dropped: 24% slower at 1M rows,
// no faster at 8M.
static int pipe_mode() {
  const char* e = std::getenv("CNF_SGPR_PIPE");
  if (e && e[0] >= '0' && e[0] <= '2') return e[0] - '0';
  return 2;
}
static bool pipe_on() { return pipe_mode() != 0; }
// A/B switch CNF_SGPR_PRIO (default on): s_setprio by tiles remaining on the
// persistent grid.  The SIMD's oldest-first arbitration otherwise finishes
// blocks far apart (tools/timeline.py: 97..231 us at 8M rows) and idles
// through the tail; measured -4 % at 8M rows, neutral at 1M.  (Non-temporal
// output stores were measured too: +27 % at 1M, dropped.)
static bool prio_on() {
  const char* e = std::getenv("CNF_SGPR_PRIO");
  return !(e && e[0] == '0');
}

static size_t lds_bytes(const Shape& s, bool pipe) {
  size_t lds = (size_t)kRW * kRows * s.D * 4;
  if (lds < (size_t)3 * kRows * 4 + 4 * 65) lds = (size_t)3 * kRows * 4 + 4 * 65;
  return lds;
}

static int resident(KFn fn, size_t lds) {
  static std::mutex mu;
  static std::unordered_map<const void*, int> cache;
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find((const void*)fn);
  if (it != cache.end()) return it->second;
  int n = 0, dev = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, kRows, lds) != hipSuccess || n < 1)
    n = 1;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus < 1)
    cus = 256;
  cache[(const void*)fn] = n * cus;
  return n * cus;
}

static KFn pick(const SEntry* e, const Shape& s, bool inverse, bool pipe) {
  return e->fn[pipe ? pipe_mode() : 0][s.scale ? 1 : 0][inverse ? 1 : 0];
}

static int64_t blocks_dir(const Shape& s, int64_t B, bool inverse) {
  const int64_t ntiles = (B + kRW * kRows - 1) / (kRW * kRows);
  const SEntry* e = find(s);
  if (!e || !pipe_on()) return ntiles;
  int cap = resident(pick(e, s, inverse, true), lds_bytes(s, true));
  if (const char* g = std::getenv("CNF_SGPR_GRID")) {  // experiment: fixed grid cap
    const int n = std::atoi(g);
    if (n > 0) cap = n;
  }
  if (ntiles <= cap) return ntiles;
  // balanced: the smallest grid that still gives every block the same tile
  // count (1M rows: 2,048 tiles on 1,024 blocks x 2, not 1,280 blocks x 1-2)
  // (measured slower: 4 waves/SIMD hide less than 5, so it stays opt-in)
  const char* b = std::getenv("CNF_SGPR_BAL");  // A/B switch: 1 = balanced grid
  if (!(b && b[0] == '1')) return cap;
  const int64_t per = (ntiles + cap - 1) / cap;
  return (ntiles + per - 1) / per;
}

int64_t sgpr_blocks(const Shape& s, int64_t B) { return blocks_dir(s, B, false); }

int sgpr_run(const Shape& s, const void* prepared, const float* in, float* out, float* ld,
             float* all, int64_t B, bool inverse, hipStream_t st, const int64_t* y,
             float* loss_ws, int kind, float det, float* loss_terms) {
  const SEntry* e = find(s);
  if (!e || !s.sp_ok || all) return CNF_ERR_UNSUPPORTED;  // every-layer outputs: k_valu
  if (B == 0) return CNF_OK;
  const char* base = static_cast<const char*>(prepared);
  const int32_t* fwd_q = reinterpret_cast<const int32_t*>(base);
  const int32_t* inv_q = fwd_q + s.L * s.D;
  const int32_t* flags = inv_q + s.L * s.D;
  const float* W = reinterpret_cast<const float*>(base + idx_bytes(s)) + s.sp_region;
  auto al = [](const void* p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  const int vec = al(in) && al(out) && al(all);
  // the inverse takes the persistent LDS-DMA form too since the weight loads became
  // compiler-visible (118 VGPRs, 4 waves/SIMD, no spills): -8 % on cfg5.
  // A/B switch CNF_SGPR_INV_PIPE=0 keeps one tile per block.
  const char* ip = std::getenv("CNF_SGPR_INV_PIPE");
  const bool pipe = pipe_on() && (!inverse || !(ip && ip[0] == '0'));
  KFn fn = pick(e, s, inverse, pipe);
  const int64_t nblk = pipe ? blocks_dir(s, B, inverse) : (B + kRW * kRows - 1) / (kRW * kRows);
  const size_t lds = lds_bytes(s, pipe);
  // one-launch loss hand-off on the persistent grid (workspace ticket word,
  // zeroed by the caller once; the last block resets it)
  const char* lt = std::getenv("CNF_LOSS_TICKET");
  const bool fused = loss_ws && pipe && lt && lt[0] == '1';  // measured slower: off
  hipLaunchKernelGGL(fn, dim3((unsigned)nblk), dim3(kRows), lds, st, W, inverse ? inv_q : fwd_q,
                     flags, in, out, ld, all, B, s.L, prio_on() ? 1 : 0, 0,
                     s.any_perm ? 1 : 0, vec,
                     y, loss_ws ? loss_ws + 4 : nullptr, kind, det,
                     fused ? reinterpret_cast<unsigned*>(loss_ws) : nullptr, loss_terms);
  if (loss_ws && !fused) reduce_partials(loss_ws + 4, (int)nblk, 4, 0, nullptr, loss_terms, st);
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    set_hip_error(err);
    return CNF_ERR_HIP;
  }
  return CNF_OK;
}

}  // namespace cnf

#ifdef CNF_TIMELINE
extern "C" int cnf_diag_timeline(unsigned long long* host, int n) {
  if (n > 4096 * 4) n = 4096 * 4;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(cnf_tl), n * 8, 0, hipMemcpyDeviceToHost) ==
                 hipSuccess
             ? n
             : -1;
}
#endif
