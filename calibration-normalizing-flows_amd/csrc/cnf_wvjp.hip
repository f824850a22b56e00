// Reverse mode for the MFMA family (every shape outside the VALU tables: D > 16,
// or wider / deeper conditioners): cnf_vjp / cnf_loss_vjp for cfg4-class flows.
//
// Replaces autograd of flows/flows.py:101-112 (NvpCouplingLayer.forward),
// flows/utils.py:26-31 (MLP.forward) and the calibrator losses
// (calibrators.py:287-291, run_experiment3D.py:102-107) for these shapes.
//
// Unlike k_vjp2 (a lane owns two rows through all L layers), a wide conditioner
// (cfg4: three 100-wide Linears per net, 12 layers, 727 K parameters) does not
// fit a row-resident sweep: its weight gradients are GEMMs whose reduction
// dimension is the batch.  So the reverse mode runs layer at a time over the
// whole batch, every product on v_mfma_f32_32x32x2_f32 (exact f32):
//
//   forward   per layer: the conditioner Linears (one launch per Linear, both
//             nets as grid.z; bias + ReLU fused into the epilogue), then the
//             coupling update + flip/permutation gather + log-det (one wave per
//             row).  Every layer's output is stashed (HBM: 288 GB leaves room),
//             so no inverse is needed.
//   seed      the loss (softmax-NLL / CE and its gradient) or the caller's
//             upstream gradients, per row; loss sums in fixed block order.
//   backward  per layer, last first: recompute the conditioner activations
//             from the stashed input, back through the coupling update (one
//             wave per row), back through the Linears (G_{k-1} = (G_k W_k) *
//             relu'(H_{k-1}); the first Linear's input gradient of both nets
//             is added into the conditioning half in one launch), then ONE
//             launch computing every Linear's weight and bias gradient as
//             G_k^T [H_{k-1} | 1] over row blocks (per-block partials summed
//             in block order: deterministic).
//
// Activation layout (workspace, row-major, every leading dimension a multiple
// of 8 floats, so A panels load as float4 and a panel's 8-wide groups never
// leave the row):
//   stash row  [x_C (DC) | 1 | 0 pad to Cp][x_T (DT) | 0 pad to DTp]  (Dp floats)
//              conditioning half first: the first Linear's operand starts the
//              row, and its ones column gives the bias gradient for free;
//   H_k row    [relu(h) (units) | 1 | 0 pad]   (Hp_k floats);
//   G_k row    [grad (nout) | 0 pad]           (Gp_k floats);
//   gradients of the layer outputs stay in the caller's natural [B][D] order.
// Pad columns are written (zeros / ones), never left uninitialised: the GEMMs
// read them and multiply them by zero weight rows.
//
// Every launch is a plain kernel on the caller's stream; no host sync.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "cnf_internal.h"

namespace cnf {
namespace {

using f16v = __attribute__((ext_vector_type(16))) float;
using f4 = __attribute__((ext_vector_type(4))) float;

constexpr int kBN = 64;      // output columns per GEMM block (2 MFMA tiles of 32)
constexpr int kKC = 128;     // reduction chunk a wave holds in registers (16 x float4)

inline int r8(int n) { return (n + 7) & ~7; }

enum Epi { kEpiBias = 0, kEpiBiasRelu = 1, kEpiMask = 2, kEpiAdd = 3 };

// C[m][n] = epi(sum_k A[m][k] B(k, n)); B(k, n) = Bw[n*ldb + k] (BT: a Linear's
// forward, W[out][in]) or Bw[k*ldb + n] (its transpose product, back-prop).
// Columns N <= n < ldw are pad: 1 at n == N when ones, else 0.
struct GemmJob {
  const float* A;
  const float* Bw;
  const float* A2;    // PAIR: C = A Bw + A2 Bw2 (both nets into one output)
  const float* Bw2;
  const float* bias;  // [N]        kEpiBias, kEpiBiasRelu
  const float* mask;  // [M][ldm]   kEpiMask: C *= (mask > 0), relu'
  float* C;
  int64_t lda, lda2, ldm, ldc;
  int ldb, ldb2, N, K, ldw, ones;
  int act;  // hidden activation of this net: 1 ReLU, 2 tanh (legacy s-net, CNF_OPT_S_TANH)
  int zlt;  // kEpiAdd: columns n < zlt add 0 * v (strict: the mask's zero columns, where
            // autograd's grad * mask keeps a NaN / inf gradient as NaN)
};
struct GemmArgs {
  GemmJob job[2];  // one per conditioner net (grid.z)
  int64_t M;
  int ny;          // column blocks; grid.x = row groups (a multiple of 8) x ny
};

// A's reduction chunk [kc, kc + 128) of one 32-row panel (lane: row r, half
// h): group g holds k = kc + 8g + 4h .. +3, one float4.  Rows past M read the
// last row (those outputs are never stored).  Leading dimensions are padded
// to 8 with written pad (zeros / the ones column), so the groups covering K
// stay inside the row and meet zero weight rows past K; a group past the row
// (only in a chunk's unused tail) reads a clamped in-row address.  No lane branches, no use of a
// loaded value before the MFMAs: the loads stay in flight.
// Buffer loads from a descriptor based at the panel's first row (wave-uniform,
// scalar arithmetic) with ONE per-lane byte offset: group g's 32 g bytes fold
// into the instruction's immediate offset, so the 16 loads cost no vector
// address arithmetic.  Groups past the row read the next row's floats (never
// used: they meet no MFMA); past the matrix's last row the descriptor's range
// check returns zeros.
__device__ __forceinline__ void load_panel(f4 (&a)[16], const float* __restrict__ A, int64_t lda,
                                           int64_t row0, int64_t M, int r, int kc, int h) {
  const int64_t rows = M - row0;  // rows left in the matrix from the panel's first
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(A + row0 * lda), 0,
      (int)std::min<int64_t>(rows * lda * 4, 0x7fffffff), 0x00020000);
  const int rr = r < rows ? r : (int)rows - 1;  // rows past M read the last row
  const int off = (rr * (int)lda + kc + 4 * h) * 4;
#pragma unroll
  for (int g = 0; g < 16; ++g)
    a[g] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 32 * g, 0, 0));
}

// acc[c] += A_panel . W[kc.., c-th 32 columns] for the chunk's ng groups; the
// LDS reads of group g+1 are issued before group g's MFMAs.  In step e of
// group g lane half h supplies k = 8g + 4h + e for A and for B alike (a
// permuted summation order, the same products).
template <int NC>
__device__ __forceinline__ void panel_mfma(f16v (&acc)[4], const f4 (&a)[16], const float* Wq,
                                           int ST, int kc, int ng, int r, int h) {
  float b[2][4][NC];  // ping-pong by group parity: no register copies
  auto ldb = [&](int g, float (&bb)[4][NC]) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float* wrow = Wq + (kc + 8 * g + 4 * h + e) * ST + r;
#pragma unroll
      for (int c = 0; c < NC; ++c) bb[e][c] = wrow[c * 32];
    }
  };
  ldb(0, b[0]);
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    if (g < ng) {
      if (g + 1 < ng) ldb(g + 1, b[(g + 1) & 1]);
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int c = 0; c < NC; ++c)
          acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[g][e], b[g & 1][e][c], acc[c], 0, 0, 0);
    }
  }
}

// The GEMM: the block stages its 32*NC-column slice of the weights (both,
// PAIR) in LDS ONCE, then each wave streams 32-row panels of A straight from
// HBM into registers (16-B loads, no LDS round trip, no barrier).  64-column
// blocks keep the wave at ~124 registers and the weight slice at ~30 KB, so
// four blocks share a CU (four waves per SIMD): a wave's panel loads and
// epilogue hide under the others' MFMAs.  (A register-prefetched next panel at one wave per SIMD measured
// slower: the compiler sinks the prefetch back next to its MFMAs.)  LDS row
// stride 32*NC + 8 puts the two lane halves' rows (4 apart)
// on disjoint banks.
template <bool BT, int EPI, bool PAIR, int NC>
__global__ __launch_bounds__(256, PAIR ? 3 : 4) void k_wgemm(GemmArgs ga) {
  const GemmJob& j = ga.job[blockIdx.z];
  // XCD-aware block order: consecutive block ids go to the 8 XCDs in turn, so
  // the ny column blocks of one row group get ids 8 apart -- the same XCD,
  // dispatched back to back -- and the second read of each A panel hits that
  // XCD's L2 instead of HBM (round 2's (x, y) grid read A once per column
  // block from HBM)
  const int bx = (int)blockIdx.x, xcd = bx & 7, q8 = bx >> 3;
  const int by = q8 % ga.ny, rg = (q8 / ga.ny) * 8 + xcd;
  extern __shared__ __attribute__((aligned(16))) float Ws[];
  const int t = threadIdx.x, lane = t & 63, r = lane & 31, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int n0 = by * kBN, N = j.N, K = j.K;
  constexpr int Nt = NC * 32, ST = Nt + 8;
  const int Kp = (K + 7) & ~7;
  // weight slice -> LDS, 8 loads in flight per thread (a dependent load-store
  // loop would pay the full memory latency per element)
#pragma unroll
  for (int q = 0; q < (PAIR ? 2 : 1); ++q) {
    const float* Bw = q ? j.Bw2 : j.Bw;
    const int ldb = q ? j.ldb2 : j.ldb;
    float* dst = Ws + q * Kp * ST;
    const int total = Kp * Nt;
    for (int i0 = 0; i0 < total; i0 += 256 * 8) {
      float v[8];
      int at[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u * 256 + t;
        int k, n;
        if (BT) {
          k = i % Kp;
          n = i / Kp;
        } else {
          n = i % Nt;
          k = i / Nt;
        }
        const int nn = n0 + n;
        const bool ok = i < total && k < K && nn < N;
        const int64_t src = ok ? (BT ? (int64_t)nn * ldb + k : (int64_t)k * ldb + nn) : 0;
        v[u] = Bw[src];
        v[u] = ok ? v[u] : 0.f;
        at[u] = i < total ? k * ST + n : -1;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (at[u] >= 0) dst[at[u]] = v[u];
    }
  }
  __syncthreads();
  const int64_t M = ga.M, panels = (M + 31) >> 5,
                stride = (int64_t)(gridDim.x / ga.ny) * 4;  // row groups x 4 waves
  // a lane's output columns are fixed for the whole launch: its biases are
  // loaded once, not after each panel's stores (j.bias may alias j.C as far as
  // the compiler knows, which would hold every panel's bias load behind them)
  float bias_c[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int n = n0 + c * 32 + r;
    bias_c[c] = (EPI == kEpiBias || EPI == kEpiBiasRelu) && n < N ? j.bias[n] : 0.f;
  }
  // The epilogue through buffer operations on descriptors based at the
  // panel's first row: a lane's offset (row 4h, its column) is fixed, each of
  // its 16 rows adds a wave-uniform scalar offset -- no per-element vector
  // address arithmetic or row guard on a full panel.  The descriptor's range
  // check covers only the VGPR offset (+ immediate), never the scalar one, so
  // the batch's ragged last panel moves each row's offset into the VGPR
  // operand: its rows past M then fall outside the range (loads read 0,
  // stores are dropped) instead of landing past the end of C.  The epilogue's
  // operands (relu' source h, or the C being added to) are all loaded before
  // the first store: j.mask / j.C may alias the output as far as the compiler
  // knows, so loads interleaved with the stores would each pay a full memory
  // round trip.
  auto rsrc_rows = [&](const float* base, int64_t ld, int64_t m0) {
    return __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(base + m0 * ld), 0,
        (int)std::min<int64_t>((M - m0) * ld * 4, 0x7fffffff), 0x00020000);
  };
  // byte offsets of row q of a lane's 16 (rows (q & 3) + 8 (q >> 2) past the
  // lane's 4h) as (VGPR part, scalar part): the scalar part on full panels,
  // all of it in the VGPR on the ragged one (see above)
  auto row_off = [](bool full, int voff, int q, int ld) {
    const int so = ((q & 3) + 8 * (q >> 2)) * ld * 4;
    return full ? int2{voff, so} : int2{voff + so, 0};
  };
  auto epilogue = [&](const f16v (&acc)[4], int64_t m0) {
    const bool full = m0 + 32 <= M;  // wave-uniform
    float pre[NC][16];
    if constexpr (EPI == kEpiMask || EPI == kEpiAdd) {
      const int64_t lds = EPI == kEpiMask ? j.ldm : j.ldc;
      const auto prs = rsrc_rows(EPI == kEpiMask ? j.mask : j.C, lds, m0);
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int n = n0 + c * 32 + r;
        const bool ok = EPI == kEpiMask ? n < N : n < j.ldw;
        const int voff = (4 * h * (int)lds + n) * 4;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int2 o = row_off(full, voff, q, (int)lds);
          const float v = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
              prs, o.x, o.y, 0));
          pre[c][q] = ok ? v : 0.f;
        }
      }
    }
    const auto crs = rsrc_rows(j.C, j.ldc, m0);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int n = n0 + c * 32 + r;
      if (n >= j.ldw) continue;
      const bool real = n < N;
      const float pad = (j.ones && n == N) ? 1.f : 0.f;
      const float b = bias_c[c];
      const int voff = (4 * h * (int)j.ldc + n) * 4;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        float v = acc[c][q];
        if constexpr (EPI == kEpiBias || EPI == kEpiBiasRelu) v += b;
        if constexpr (EPI == kEpiBiasRelu) {  // the hidden activation
          if (j.act == 2) v = tanhf(v);
          else v = v < 0.f ? 0.f : v;  // keeps NaN (torch relu)
        }
        if constexpr (EPI == kEpiMask) {  // its derivative from the stored output h
          const float hh = pre[c][q];
          v = j.act == 2 ? v * (1.f - hh * hh) : (hh <= 0.f ? 0.f : v);
          if (!real) v = 0.f;
        }
        if constexpr (EPI == kEpiAdd) v = (n < j.zlt ? 0.f * v : v) + pre[c][q];
        const int2 o = row_off(full, voff, q, (int)j.ldc);
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, real ? v : pad), crs, o.x,
                                              o.y, 0);
      }
    }
  };
  int64_t pn = (int64_t)rg * 4 + w;
  for (; pn < panels; pn += stride) {
    f16v acc[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] = f16v{};
#pragma unroll
    for (int q = 0; q < (PAIR ? 2 : 1); ++q) {
      const float* A = q ? j.A2 : j.A;
      const int64_t lda = q ? j.lda2 : j.lda;
      for (int kc = 0; kc < Kp; kc += kKC) {
        f4 a[16];
        load_panel(a, A, lda, pn * 32, M, r, kc, h);
        panel_mfma<NC>(acc, a, Ws + q * Kp * ST, ST, kc, min(16, (Kp - kc) >> 3), r, h);
      }
    }
    epilogue(acc, pn * 32);
  }
}

// Weight gradients dW = G^T [H | 1] of every (net, Linear) job of a layer over
// row blocks (per-block partials in state_dict layout, summed in block order
// afterwards: deterministic).  A block of four waves owns a 128-row x
// 128-column group of one job's dW: wave w the 32 output rows n0 = 32(4 g_n +
// w) .. +31 and EVERY column tile of the group.  The four waves therefore
// stream the SAME H rows at the same time (one HBM pass: the other three
// waves' reads hit L1 / L2) and each its own 32 G columns, so each operand
// leaves HBM once per layer.  (Round 2's one-wave blocks, one 32 x 64 tile
// each, re-read every G column per column tile and every H column per output
// tile: 2-4x the algorithmic bytes.)  In k-step s lane (i, h) reads
// G[row][n0 + i] and H[row][c0 + 32c + i] of row mr + 2s + h: 128 contiguous
// bytes per half-wave.  The next 32 rows' operands load under this chunk's
// MFMAs.  Column tiles past the job (nct < 4) are skipped by wave-uniform
// branches; out-of-range outputs read clamped addresses and are never written;
// only the batch's ragged end masks rows.
struct DwJob {
  const float* G;
  const float* H;
  int64_t ldg, ldh;
  int64_t woff, boff;  // float offsets of W[0][in_off] and b[0] in the layer record
  int wld, N, K, tiles_c;  // tiles_c: 32-column tiles of [H | 1] (K + 1 columns)
  int cstep;           // +1, or -1 when the kernel's input columns run reversed (legacy)
  int rrev;            // output rows reversed (legacy): row n is parameter row N_full-1-n
  int nfull;
  int gcl, hcl;        // last G / H column a lane may read (k_wdw16)
  int slot;            // k_wdw16: G and H columns in slot order (the fused sweeps' layout:
                       // column c holds unit slot_unit(c)), natural otherwise
};
struct DwArgs {
  DwJob job[2 * kMaxLin];
  float* partials;  // [nkb][PS]
  int64_t M, rows, PS;
};

// CNF_WDW16 (default 1): the layer-at-a-time weight gradients on k_wdw16's
// 16x16x4 tiles; 0 compiles and runs k_wdw's 32x32x2 predecessor instead
// (A/B builds only: make ab ABSRC=cnf_wvjp DEFS=-DCNF_WDW16=0)
#ifndef CNF_WDW16
#define CNF_WDW16 1
#endif
#if !CNF_WDW16
constexpr int kDwCT = 4;  // column tiles per wave (128 columns)

__global__ __launch_bounds__(256, 3) void k_wdw(DwArgs da) {
  // the job's fields once, into scalar registers (a reference into the
  // argument block indexed by blockIdx.y reloads every field at every use)
  const DwJob j = da.job[blockIdx.y];
  const int lane = threadIdx.x & 63, i = lane & 31, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nsub = (j.N + 31) >> 5, ncg = (j.tiles_c + kDwCT - 1) / kDwCT;
  const int gn = (int)blockIdx.z / ncg, cg = (int)blockIdx.z % ncg;
  const int ns = gn * 4 + w;
  if (gn * 4 >= nsub || ns >= nsub) return;  // no __syncthreads below: waves may leave
  const int nct = min(kDwCT, j.tiles_c - cg * kDwCT);
  const int n0 = ns * 32, c0 = cg * 32 * kDwCT;
  const int64_t r0 = (int64_t)blockIdx.x * da.rows;
  const int64_t r1 = min(da.M, r0 + da.rows);
  if (r0 >= r1) return;
  // operand addresses: buffer loads from a wave-uniform descriptor based at
  // the chunk's first row (scalar arithmetic), a per-lane 32-bit byte offset
  // fixed for the whole launch (row h of the pair, column n0 + i / c0 + 32c +
  // i, clamped in-row) and a scalar offset per row pair -- no per-load vector
  // address arithmetic
  const int ldg = (int)j.ldg, ldh = (int)j.ldh;
  const int goff = (h * ldg + min(n0 + i, j.N - 1)) * 4;
  int hoff[kDwCT];
#pragma unroll
  for (int c = 0; c < kDwCT; ++c) hoff[c] = (h * ldh + min(c0 + 32 * c + i, ldh - 1)) * 4;
  // 16-row chunks (8 MFMA k-steps) in two operand sets used in turn: the next
  // chunk's loads are issued before this chunk's MFMAs without register copies
  constexpr int KS = 8;
  auto load = [&](int64_t mr, float (&a)[KS], float (&b)[kDwCT][KS]) {
    const auto gr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(j.G + mr * ldg), 0,
                                                      0x7fffffff, 0x00020000);
    const auto hr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(j.H + mr * ldh), 0,
                                                      0x7fffffff, 0x00020000);
#pragma unroll
    for (int s = 0; s < KS; ++s)
      a[s] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(gr, goff, 2 * s * ldg * 4, 0));
#pragma unroll
    for (int c = 0; c < kDwCT; ++c)
      if (c < nct) {
#pragma unroll
        for (int s = 0; s < KS; ++s)
          b[c][s] = __builtin_bit_cast(
              float, __builtin_amdgcn_raw_buffer_load_b32(hr, hoff[c], 2 * s * ldh * 4, 0));
      }
  };
  auto mfmas = [&](f16v (&acc)[kDwCT], const float* a, const float (*b)[KS], int ks) {
#pragma unroll
    for (int c = 0; c < kDwCT; ++c)
      if (c < nct) {
#pragma unroll
        for (int s = 0; s < ks; ++s)
          acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], b[c][s], acc[c], 0, 0, 0);
      }
  };
  f16v acc[kDwCT];
#pragma unroll
  for (int c = 0; c < kDwCT; ++c) acc[c] = f16v{};
  const int64_t rfull = r0 + (r1 - r0) / 16 * 16;  // rows in whole chunks
  if (rfull > r0) {
    float a0[KS], b0[kDwCT][KS], a1[KS], b1[kDwCT][KS];
    load(r0, a0, b0);
    for (int64_t mr = r0;; mr += 32) {
      const bool more1 = mr + 16 < rfull;
      if (more1) load(mr + 16, a1, b1);
      __builtin_amdgcn_sched_barrier(0);
      mfmas(acc, a0, b0, KS);
      if (!more1) break;
      const bool more2 = mr + 32 < rfull;
      if (more2) load(mr + 32, a0, b0);
      __builtin_amdgcn_sched_barrier(0);
      mfmas(acc, a1, b1, KS);
      if (!more2) break;
    }
  }
  if (rfull < r1) {  // the batch's ragged end: rows past r1 contribute zero
    float a[KS], b[kDwCT][KS];
    const float* G = j.G;
    const float* H = j.H;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int64_t row = rfull + 2 * s + h;
      const bool ok = row < r1;
      const int64_t rr = ok ? row : r1 - 1;
      a[s] = ok ? G[rr * ldg + min(n0 + i, j.N - 1)] : 0.f;
#pragma unroll
      for (int c = 0; c < kDwCT; ++c) b[c][s] = H[rr * ldh + min(c0 + 32 * c + i, ldh - 1)];
    }
    mfmas(acc, a, b, KS);
  }
  float* out = da.partials + (int64_t)blockIdx.x * da.PS;
#pragma unroll
  for (int c = 0; c < kDwCT; ++c) {
    const int k = c0 + c * 32 + i;
    if (c >= nct || k > j.K) continue;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int nn = n0 + (q & 3) + 8 * (q >> 2) + 4 * h;
      if (nn >= j.N) continue;
      const int pr = j.rrev ? j.nfull - 1 - nn : nn;  // parameter row
      if (k < j.K) out[j.woff + (int64_t)pr * j.wld + (int64_t)j.cstep * k] = acc[c][q];
      else out[j.boff + pr] = acc[c][q];
    }
  }
}

#endif  // !CNF_WDW16

// The same weight gradients on v_mfma_f32_16x16x4f32 tiles (the same 64
// FLOP/clk/SIMD as 32x32x2): a wave still owns 32 output rows, and up to 112
// columns, as 16 x 16 tiles, so a job's padding is to the next 16 instead of 32 --
// N = 100 needs 7 row tiles (112) instead of 4 x 32 (128), the 101 columns
// of [H | 1] 7 column tiles (112) instead of 128: the (100, 101) job issues
// 49 tiles' MFMAs instead of 64, a cfg4 layer 18 % fewer in all.  Operand
// loads per 16 rows are unchanged (K-step s: lane (i, q) reads G[row 4s + q]
// [n + i] and H[row 4s + q][c + i], 64 contiguous bytes per quarter-wave).
#ifndef CNF_DW16_CT
#define CNF_DW16_CT 7
#endif
// 16-column tiles per wave (7: 112 columns, [H | 1] of a 100-wide layer in one
// block; 4: two blocks of 64 + 48 columns, half the accumulators, four waves
// per SIMD)
constexpr int kDw16CT = CNF_DW16_CT;
#ifndef CNF_DW16_KS
#define CNF_DW16_KS 4
#endif
// MFMA k-steps (of 4 rows) per operand set: 4 (16-row chunks, 149 VGPRs, 3
// waves per SIMD) or 2 (8-row chunks, 4 waves per SIMD)
constexpr int kDw16KS = CNF_DW16_KS;

// unit of slot c in a 16-slot tile (cnf_wide16.hip's q-major fill; an involution)
__device__ __forceinline__ int slot_unit(int c) {
  return 16 * (c >> 4) + 4 * (c & 3) + ((c & 15) >> 2);
}

__global__ __launch_bounds__(256, (kDw16CT <= 4 || kDw16KS <= 2) ? 4 : 3) void k_wdw16(DwArgs da) {
  const DwJob j = da.job[blockIdx.y];
  const int lane = threadIdx.x & 63, i = lane & 15, kq = lane >> 4;
  // (rotating the 32-row group a wave takes by the row block, to spread the
  // short and idle waves of N = 100 / 50 jobs over the SIMDs, measured no
  // change: 14.57 vs 14.60 ms per cfg4 step)
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tiles16 = (j.K + 1 + 15) >> 4;
  const int nsub = (j.N + 31) >> 5, ncg = (tiles16 + kDw16CT - 1) / kDw16CT;
  const int gn = (int)blockIdx.z / ncg, cg = (int)blockIdx.z % ncg;
  const int ns = gn * 4 + w;
  if (gn * 4 >= nsub || ns >= nsub) return;  // no __syncthreads below: waves may leave
  const int n0 = ns * 32, c0 = cg * 16 * kDw16CT;
  const int nrs = n0 + 16 < j.N ? 2 : 1;  // 16-row tiles of this wave (wave-uniform)
  const int nct = min(kDw16CT, tiles16 - cg * kDw16CT);
  const int64_t r0 = (int64_t)blockIdx.x * da.rows;
  const int64_t r1 = min(da.M, r0 + da.rows);
  if (r0 >= r1) return;
  const int ldg = (int)j.ldg, ldh = (int)j.ldh;
  // operand addressing.  Natural rows: element (r, c) at r * ld + c, k-step s
  // 4 rows (4 ld floats) on.  Slot jobs read the fused sweeps' wave-tiled
  // arrays (cnf_internal.h): (r, c) at (r >> 5) * 32 ld + (c >> 4) * 512 +
  // ((r >> 4) & 1) * 256 + (r & 15) * 16 + (c & 15), k-step s 64 floats on
  // (a 16-row chunk never leaves its row group).  Columns past a part clamp
  // to its last column (tile).
  int goff[2], hoff[kDw16CT];
  if (j.slot) {
#pragma unroll
    for (int t = 0; t < 2; ++t) goff[t] = (min((n0 >> 4) + t, j.gcl >> 4) * 512 + kq * 16 + i) * 4;
#pragma unroll
    for (int c = 0; c < kDw16CT; ++c)
      hoff[c] = (min((c0 >> 4) + c, j.hcl >> 4) * 512 + kq * 16 + i) * 4;
  } else {
#pragma unroll
    for (int t = 0; t < 2; ++t) goff[t] = (kq * ldg + min(n0 + 16 * t + i, j.gcl)) * 4;
#pragma unroll
    for (int c = 0; c < kDw16CT; ++c) hoff[c] = (kq * ldh + min(c0 + 16 * c + i, j.hcl)) * 4;
  }
  const int gstep = j.slot ? 256 : 16 * ldg, hstep = j.slot ? 256 : 16 * ldh;  // bytes per k-step
  auto chunk = [&](const float* P, int64_t ld, int64_t mr) {
    return j.slot ? P + (mr >> 5) * 32 * ld + ((mr >> 4) & 1) * 256 + (mr & 15) * 16 : P + mr * ld;
  };
  auto elt = [&](const float* P, int64_t ld, int64_t r, int c, int cl) {
    return j.slot ? P[(r >> 5) * 32 * ld + min(c >> 4, cl >> 4) * 512 + ((r >> 4) & 1) * 256 +
                      (r & 15) * 16 + (c & 15)]
                  : P[r * ld + min(c, cl)];
  };
  // chunks of 4 KS rows (KS MFMA k-steps of 4 rows) in two operand sets used in turn
  constexpr int KS = kDw16KS, CH = 4 * KS;
  auto load = [&](int64_t mr, float (&a)[2][KS], float (&b)[kDw16CT][KS]) {
    const auto gr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(chunk(j.G, ldg, mr)), 0,
                                                      0x7fffffff, 0x00020000);
    const auto hr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(chunk(j.H, ldh, mr)), 0,
                                                      0x7fffffff, 0x00020000);
#pragma unroll
    for (int t = 0; t < 2; ++t)
      if (t < nrs) {
#pragma unroll
        for (int s = 0; s < KS; ++s)
          a[t][s] = __builtin_bit_cast(
              float, __builtin_amdgcn_raw_buffer_load_b32(gr, goff[t], s * gstep, 0));
      }
#pragma unroll
    for (int c = 0; c < kDw16CT; ++c)
      if (c < nct) {
#pragma unroll
        for (int s = 0; s < KS; ++s)
          b[c][s] = __builtin_bit_cast(
              float, __builtin_amdgcn_raw_buffer_load_b32(hr, hoff[c], s * hstep, 0));
      }
  };
  // k-step outermost: consecutive MFMAs update different accumulators (a
  // dependent 16x16x4 has 40 cycles of latency against 32 of issue)
  auto mfmas = [&](f4 (&acc)[2][kDw16CT], const float (*a)[KS], const float (*b)[KS]) {
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int t = 0; t < 2; ++t)
        if (t < nrs) {
#pragma unroll
          for (int c = 0; c < kDw16CT; ++c)
            if (c < nct)
              acc[t][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t][s], b[c][s], acc[t][c], 0, 0, 0);
        }
  };
  f4 acc[2][kDw16CT];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int c = 0; c < kDw16CT; ++c) acc[t][c] = f4{};
  const int64_t rfull = r0 + (r1 - r0) / CH * CH;  // rows in whole chunks
  if (rfull > r0) {
    float a0[2][KS], b0[kDw16CT][KS], a1[2][KS], b1[kDw16CT][KS];
    load(r0, a0, b0);
    for (int64_t mr = r0;; mr += 2 * CH) {
      const bool more1 = mr + CH < rfull;
      if (more1) load(mr + CH, a1, b1);
      __builtin_amdgcn_sched_barrier(0);
      mfmas(acc, a0, b0);
      if (!more1) break;
      const bool more2 = mr + 2 * CH < rfull;
      if (more2) load(mr + 2 * CH, a0, b0);
      __builtin_amdgcn_sched_barrier(0);
      mfmas(acc, a1, b1);
      if (!more2) break;
    }
  }
  if (rfull < r1) {  // the batch's ragged end: rows past r1 contribute zero
    float a[2][KS], b[kDw16CT][KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int64_t row = rfull + 4 * s + kq;
      const bool ok = row < r1;
      const int64_t rr = ok ? row : r1 - 1;
#pragma unroll
      for (int t = 0; t < 2; ++t) a[t][s] = ok ? elt(j.G, ldg, rr, n0 + 16 * t + i, j.gcl) : 0.f;
#pragma unroll
      for (int c = 0; c < kDw16CT; ++c) b[c][s] = elt(j.H, ldh, rr, c0 + 16 * c + i, j.hcl);
    }
    mfmas(acc, a, b);
  }
  // lane (i, kq), register q of tile (t, c): dW row n0 + 16 t + 4 kq + q, column c0 + 16 c + i
  // (slot jobs: the units of those slots)
  float* out = da.partials + (int64_t)blockIdx.x * da.PS;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    if (t >= nrs) continue;
#pragma unroll
    for (int c = 0; c < kDw16CT; ++c) {
      const int kc = c0 + c * 16 + i;
      const int k = j.slot ? slot_unit(kc) : kc;
      if (c >= nct || k > j.K) continue;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int nc = n0 + 16 * t + 4 * kq + q;
        const int nn = j.slot ? slot_unit(nc) : nc;
        if (nn >= j.N) continue;
        const int pr = j.rrev ? j.nfull - 1 - nn : nn;  // parameter row
        if (k < j.K) out[j.woff + (int64_t)pr * j.wld + (int64_t)j.cstep * k] = acc[t][c][q];
        else out[j.boff + pr] = acc[t][c][q];
      }
    }
  }
}

// The fused sweeps' weight gradients (slot jobs on the wave-tiled G / H
// arrays, cnf_internal.h) with each 32-row block's operand tiles staged in LDS:
// in the wave-tiled layout a block's G part and H part are contiguous runs of
// 2 KiB tiles, so the four waves copy them by LDS-DMA (global_load_lds, 1 KiB
// per wave-instruction, no registers) into one of two stages while computing
// the other, and every wave reads its MFMA operands from LDS -- H once per
// block instead of once per wave.  Wave w takes the job's row tiles w and
// w + 4 (of 7 for N = 100, of 4 for N = 50) over every column tile.  Rows past
// the batch inside the last 32-row block are padding the sweeps wrote with
// exact zeros in G (zero upstream gradients), so whole blocks are summed.
// Compile-time tile counts (NTG G tiles, NTH H tiles, NR row tiles for this
// wave), so the k-step body is straight-line MFMAs on LDS operands.
template <int NTG, int NTH, int NR>
__device__ __forceinline__ void wdwg_chunks(const DwJob& j, float* sm, int w, int lane, int64_t r0,
                                            int nch, f4 (&acc)[2][8]) {
  constexpr int TPC = NTG + NTH;
  const int64_t ldg = j.ldg, ldh = j.ldh;
  auto dma = [&](int c, int stg) {
    const float* gsrc = j.G + ((r0 >> 5) + c) * 32 * ldg;
    const float* hsrc = j.H + ((r0 >> 5) + c) * 32 * ldh;
    float* dst = sm + stg * TPC * 512;
#pragma unroll
    for (int k0 = 0; k0 < 2 * TPC; k0 += 4) {  // 1 KiB pieces; piece k0 + w is this wave's
      const int k = k0 + w;
      if (k < 2 * TPC) {
        const float* src = k < 2 * NTG ? gsrc + k * 256 : hsrc + (k - 2 * NTG) * 256;
        __builtin_amdgcn_global_load_lds(const_cast<float*>(src) + lane * 4, dst + k * 256, 16, 0, 0);
      }
    }
  };
  dma(0, 0);
  for (int c = 0; c < nch; ++c) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of chunk c
    __syncthreads();  // everyone's pieces landed; everyone is done with chunk c - 1
    if (c + 1 < nch) dma(c + 1, (c + 1) & 1);
    const float* S = sm + (c & 1) * TPC * 512 + lane;
#pragma unroll
    for (int s = 0; s < 8; ++s) {  // 4 rows per k-step: row 4s + kq of the 32-row block
      float a[NR > 0 ? NR : 1], b[NTH];
#pragma unroll
      for (int t = 0; t < NR; ++t) a[t] = S[(w + 4 * t) * 512 + s * 64];
#pragma unroll
      for (int q = 0; q < NTH; ++q) b[q] = S[(NTG + q) * 512 + s * 64];
#pragma unroll
      for (int t = 0; t < NR; ++t)
#pragma unroll
        for (int q = 0; q < NTH; ++q)
          acc[t][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t], b[q], acc[t][q], 0, 0, 0);
    }
  }
}

// The same chunk loop with the job's (row tile, column tile) pairs dealt to
// the four waves round-robin (pair p = NTH t + c to wave p % 4) instead of
// whole row tiles: a 7-row-tile job gave waves 0-2 two row tiles and wave 3
// one (each block's fourth SIMD half idle), a 1-row-tile job all its work to
// wave 0.  A wave reads the operand tiles its pairs touch (unused reads are
// dropped by the compiler) and writes its own cells.
#ifndef CNF_WDWG_RR
#define CNF_WDWG_RR 1
#endif
// A/B timing only (wrong results): 1 = no MFMAs, 2 = no operand DMA (the
// MFMAs run on whatever the LDS stages hold)
template <int NTG, int NTH, int W>
__device__ __forceinline__ void wdwg_rr(const DwJob& j, const DwArgs& da, float* sm, int lane,
                                        int64_t r0, int nch) {
  constexpr int TPC = NTG + NTH, NPJ = NTG * NTH;
  constexpr int NP = NPJ > W ? (NPJ - W + 3) / 4 : 0;  // this wave's pairs
  const int64_t ldg = j.ldg, ldh = j.ldh;
  const int i = lane & 15, kq = lane >> 4;
  f4 acc[NP > 0 ? NP : 1];
#pragma unroll
  for (int m = 0; m < NP; ++m) acc[m] = f4{};
  auto dma = [&](int c, int stg) {
    const float* gsrc = j.G + ((r0 >> 5) + c) * 32 * ldg;
    const float* hsrc = j.H + ((r0 >> 5) + c) * 32 * ldh;
    float* dst = sm + stg * TPC * 512;
#pragma unroll
    for (int k0 = 0; k0 < 2 * TPC; k0 += 4) {  // 1 KiB pieces; piece k0 + W is this wave's
      const int k = k0 + W;
      if (k < 2 * TPC) {
        const float* src = k < 2 * NTG ? gsrc + k * 256 : hsrc + (k - 2 * NTG) * 256;
        __builtin_amdgcn_global_load_lds(const_cast<float*>(src) + lane * 4, dst + k * 256, 16, 0, 0);
      }
    }
  };
  dma(0, 0);
  for (int c = 0; c < nch; ++c) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of chunk c
    __syncthreads();  // everyone's pieces landed; everyone is done with chunk c - 1
    if (c + 1 < nch) dma(c + 1, (c + 1) & 1);
    const float* S = sm + (c & 1) * TPC * 512 + lane;
#pragma unroll
    for (int s = 0; s < 8; ++s) {  // 4 rows per k-step: row 4s + kq of the 32-row block
      float a[NTG], b[NTH];
#pragma unroll
      for (int t = 0; t < NTG; ++t) a[t] = S[t * 512 + s * 64];
#pragma unroll
      for (int q = 0; q < NTH; ++q) b[q] = S[(NTG + q) * 512 + s * 64];
#pragma unroll
      for (int m = 0; m < NP; ++m) {
        const int p = W + 4 * m;
        acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[p / NTH], b[p % NTH], acc[m], 0, 0, 0);
      }
    }
  }
  // lane (i, kq), register q of pair (t, c): dW row slot 16 t + 4 kq + q,
  // column slot 16 c + i, each mapped to its unit
  float* out = da.partials + (int64_t)blockIdx.x * da.PS;
#pragma unroll
  for (int m = 0; m < NP; ++m) {
    const int p = W + 4 * m, t = p / NTH, c = p % NTH;
    const int k = slot_unit(16 * c + i);
    if (k > j.K) continue;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int nn = slot_unit(16 * t + 4 * kq + q);
      if (nn >= j.N) continue;
      if (k < j.K) out[j.woff + (int64_t)nn * j.wld + k] = acc[m][q];
      else out[j.boff + nn] = acc[m][q];
    }
  }
}

// the (G tiles, H tiles) classes with an instantiation: the weight gradients
// of k_wide16's table (cfg4: (7, 4), (7, 7), (4, 7))
#define CNF_WDWG_CLASSES(X) X(7, 4) X(7, 7) X(4, 7) X(4, 4) X(4, 2) X(4, 5) X(1, 5)
inline bool wdwg_class_ok(int ntg, int nth) {
#define CNF_WDWG_OK(A, B) if (ntg == A && nth == B) return true;
  CNF_WDWG_CLASSES(CNF_WDWG_OK)
#undef CNF_WDWG_OK
  return false;
}

__global__ __launch_bounds__(256, 2) void k_wdw16g(DwArgs da) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const DwJob j = da.job[blockIdx.y];
  const int lane = threadIdx.x & 63, i = lane & 15, kq = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ntg = (j.gcl >> 4) + 1, nth = (j.hcl >> 4) + 1;
  const int64_t r0 = (int64_t)blockIdx.x * da.rows;
  const int64_t r1 = min(da.M, r0 + da.rows);  // da.M: the batch rounded up to 32
  if (r0 >= r1) return;  // the whole block: no barrier reached
  const int nch = (int)((r1 - r0) >> 5);
  const int nr = (w < ntg ? 1 : 0) + (w + 4 < ntg ? 1 : 0);
  f4 acc[2][8];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[t][c] = f4{};
  // every wave runs the chunk loop (it copies its share and meets the
  // barriers) whatever its row-tile count
#define CNF_WDWG_RUN(A, B)                                                    \
  if (ntg == A && nth == B) {                                                 \
    if (CNF_WDWG_RR && A % 4 != 0) {                                          \
      if (w == 0) wdwg_rr<A, B, 0>(j, da, sm, lane, r0, nch);                 \
      else if (w == 1) wdwg_rr<A, B, 1>(j, da, sm, lane, r0, nch);            \
      else if (w == 2) wdwg_rr<A, B, 2>(j, da, sm, lane, r0, nch);            \
      else wdwg_rr<A, B, 3>(j, da, sm, lane, r0, nch);                        \
      return;                                                                 \
    }                                                                         \
    if (nr == 2) wdwg_chunks<A, B, 2>(j, sm, w, lane, r0, nch, acc);           \
    else if (nr == 1) wdwg_chunks<A, B, 1>(j, sm, w, lane, r0, nch, acc);      \
    else wdwg_chunks<A, B, 0>(j, sm, w, lane, r0, nch, acc);                   \
  } else
  CNF_WDWG_CLASSES(CNF_WDWG_RUN) {}
#undef CNF_WDWG_RUN
  // lane (i, kq), register q of tile (t, c): dW row slot 16 (w + 4t) + 4 kq + q,
  // column slot 16 c + i, each mapped to its unit
  float* out = da.partials + (int64_t)blockIdx.x * da.PS;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    if (t >= nr) continue;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int k = slot_unit(16 * c + i);
      if (c >= nth || k > j.K) continue;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int nn = slot_unit(16 * (w + 4 * t) + 4 * kq + q);
        if (nn >= j.N) continue;
        if (k < j.K) out[j.woff + (int64_t)nn * j.wld + k] = acc[t][c][q];
        else out[j.boff + nn] = acc[t][c][q];
      }
    }
  }
}

#ifndef CNF_WDW16G
#define CNF_WDW16G 1  // A/B: 0 runs the fused sweeps' weight gradients on k_wdw16
#endif

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Row geometry of the stash layout (see the file comment).  strict
// (cnf_desc.strict_nan): the first Linear reads the reference's whole masked
// input x_b = mask * x (0 * x_T: 0, or NaN where x_T is not finite) and the
// last Linear writes s, t for all D features, so the C part is
// [x_b (D) | 1 | pad] and raw x_j sits in the C part for j >= DT (mask 1:
// x_b = x) and in the T part for j < DT; O rows (and G of the last Linear)
// are Op = r8(D) wide instead of DTp.
struct Geo {
  int D, DT, DC, Cp, DTp, Dp, Op, strict;
  // column of RAW x_j in a stash row
  __device__ __forceinline__ int col(int i) const {
    return i < DT ? Cp + i : (strict ? i : i - DT);
  }
  // the C part's ones column
  __device__ __forceinline__ int ones() const { return strict ? D : DC; }
};

// A layer's gather table (D <= CNF_MAX_DIM ints) staged in LDS once per block:
// the row loops then index it without a dependent global load per element
// (the table lookups had put two serialized memory round trips into every
// row's update).
__device__ __forceinline__ const int32_t* stage_table(int32_t* sq, const int32_t* __restrict__ q,
                                                      int D) {
  for (int j = threadIdx.x; j < D; j += blockDim.x) sq[j] = q[j];
  __syncthreads();
  return sq;
}

// Natural [B][D] rows -> stash layout (the first layer's input).
__global__ __launch_bounds__(256) void k_wstash(const float* __restrict__ x,
                                                float* __restrict__ xs, int64_t B, Geo g) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < B; r += nw) {
    for (int c = lane; c < g.Dp; c += 64) {
      float v;
      if (g.strict && c < g.D) v = c < g.DT ? 0.f * x[r * g.D + c] : x[r * g.D + c];  // mask * x
      else if (!g.strict && c < g.DC) v = x[r * g.D + g.DT + c];
      else if (c == g.ones()) v = 1.f;
      else if (c >= g.Cp && c < g.Cp + g.DT) v = x[r * g.D + c - g.Cp];
      else v = 0.f;
      xs[r * g.Dp + c] = v;
    }
  }
}

// Coupling update of one layer (flows/flows.py:101-112), one wave per row:
//   z_i = x_i e^{s_i} + t_i (i < DT), x_i otherwise; ld += sum_i s_i;
//   out[j] = z[fq[j]] (permutation, then flip); stash layout in and out.
// strict: the reference's own op sequence over ALL features,
//   z_i = m_i x_i + (1 - m_i) (x_i e^{s_i} + t_i),  ld += sum_i (1 - m_i) s_i,
// one rounding per op, so 0 * inf = NaN at masked positions as in torch.
// A wave takes kRU rows at a time and issues every load of the group before
// the first use (lane l: columns j = l + 64q), so a wave has kRU rows of
// loads in flight instead of one row's dependent round trips.
constexpr int kRU = 4;  // rows per wave per group
// kNJ = column slots per lane, ceil(D / 64) (a template parameter, so the
// register arrays are only as wide as the row)
template <int kNJ>
__global__ __launch_bounds__(256) void k_wfwd_update(const float* __restrict__ X,
                                                     float* __restrict__ Xn, float* __restrict__ ld,
                                                     const float* __restrict__ Os,
                                                     const float* __restrict__ Ot,
                                                     const int32_t* __restrict__ fqg, int64_t B,
                                                     Geo g, int first) {
  __shared__ int32_t sq[CNF_MAX_DIM];
  const int32_t* fq = stage_table(sq, fqg, g.D);
  const int lane = threadIdx.x & 63;
  int ii[kNJ];
#pragma unroll
  for (int q = 0; q < kNJ; ++q) ii[q] = lane + 64 * q < g.D ? fq[lane + 64 * q] : 0;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * kRU; r0 < B; r0 += nw * kRU) {
    float v[kRU][kNJ], sv[kRU][kNJ], tv[kRU][kNJ], so[kRU][kNJ], ldo[kRU];
#pragma unroll
    for (int u = 0; u < kRU; ++u) {
      const int64_t r = r0 + u < B ? r0 + u : B - 1;  // past-the-end rows: loads only
      ldo[u] = first ? 0.f : ld[r];
#pragma unroll
      for (int q = 0; q < kNJ; ++q) {
        const int j = lane + 64 * q, i = ii[q];
        v[u][q] = sv[u][q] = tv[u][q] = so[u][q] = 0.f;
        if (j < g.D) {
          v[u][q] = X[r * g.Dp + g.col(i)];
          if (i < g.DT || g.strict) {
            if (Os) sv[u][q] = Os[r * g.Op + i];
            if (Ot) tv[u][q] = Ot[r * g.Op + i];
          }
        }
        if (Os && j < (g.strict ? g.D : g.DT)) so[u][q] = Os[r * g.Op + j];
      }
    }
#pragma unroll
    for (int u = 0; u < kRU; ++u) {
      const int64_t r = r0 + u;
      if (r >= B) break;
      float* zr = Xn + r * g.Dp;
      float sacc = 0.f;
#pragma unroll
      for (int q = 0; q < kNJ; ++q) {
        const int j = lane + 64 * q;
        if (j < g.D) {
          float x = v[u][q];
          if (g.strict) {  // x_b + b_1 (x e^s + t), b_1 = 1 - mask
            const float b1 = ii[q] < g.DT ? 1.f : 0.f;
            const float w = __fmul_rn(b1, __fadd_rn(__fmul_rn(x, expf(sv[u][q])), tv[u][q]));
            x = __fadd_rn(__fmul_rn(1.f - b1, x), w);
            if (j < g.DT) zr[j] = 0.f * x;  // the next layer's x_b (mask 0 here)
          } else if (ii[q] < g.DT) {
            x = __fadd_rn(__fmul_rn(x, expf(sv[u][q])), tv[u][q]);
          }
          zr[g.col(j)] = x;
        }
        sacc += g.strict && j >= g.DT ? 0.f * so[u][q] : so[u][q];
      }
      for (int c = g.ones() + lane; c < g.Cp; c += 64) zr[c] = c == g.ones() ? 1.f : 0.f;
      for (int c = g.Cp + g.DT + lane; c < g.Dp; c += 64) zr[c] = 0.f;
      sacc = wave_sum(sacc);
      if (lane == 0) ld[r] = first ? sacc : ldo[u] + sacc;
    }
  }
}

// Upstream gradient at z_L (stash layout), one wave per row, into natural
// order.  Loss kinds as k_vjp2 (cnf_vjp.hip); generic: gz (+ gz_all[L-1]) and
// gld.  Loss sums per block in fixed order: partials[block][0..2] = (loss, ce,
// ld).
__global__ __launch_bounds__(256) void k_wseed(const float* __restrict__ Z,
                                               const float* __restrict__ ld,
                                               const int64_t* __restrict__ y, int kind, float det,
                                               float grad_scale, const float* __restrict__ gz,
                                               const float* __restrict__ gz_last,
                                               const float* __restrict__ gld_in,
                                               float* __restrict__ G, float* __restrict__ gld,
                                               float* __restrict__ partials, int64_t B, Geo g) {
  __shared__ float red[4][3];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int D = g.D;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f;
  for (int64_t r = (int64_t)blockIdx.x * 4 + wv; r < B; r += nw) {
    if (kind < 0) {
      for (int j = lane; j < D; j += 64) {
        float v = gz ? gz[r * D + j] : 0.f;
        if (gz_last) v += gz_last[r * D + j];
        G[r * D + j] = v;
      }
      if (lane == 0) gld[r] = gld_in ? gld_in[r] : 0.f;
      continue;
    }
    const float* zr = Z + r * g.Dp;
    float m = -INFINITY;
    for (int j = lane; j < D; j += 64) m = fmaxf(m, zr[g.col(j)]);
    m = wave_max(m);
    float se = 0.f;
    for (int j = lane; j < D; j += 64) se += expf(zr[g.col(j)] - m);
    se = wave_sum(se);
    const float lse = m + logf(se);
    const int64_t yy = y[r];
    const bool ok = yy >= 0 && yy < D;
    const int yi = ok ? (int)yy : 0;
    const float lpy = zr[g.col(yi)] - lse;
    const float ldr = ld[r];
    float coef, ce, loss, gl;
    if (kind == CNF_LOSS_CAL) {  // -(log(softmax(z)[y] + 1e-7) + ld)
      const float py = expf(lpy);
      ce = -logf(py + 1e-7f);
      loss = ce - ldr;
      coef = py / (py + 1e-7f);
      gl = -grad_scale;
    } else {  // CE(z, y) - det * ld
      ce = -lpy;
      loss = ce - det * ldr;
      coef = 1.f;
      gl = -det * grad_scale;
    }
    if (!ok) ce = loss = coef = __builtin_nanf("");
    for (int j = lane; j < D; j += 64) {
      const float pj = expf(zr[g.col(j)] - lse);
      G[r * D + j] = grad_scale * coef * (pj - (j == yi ? 1.f : 0.f));
    }
    if (lane == 0) {
      gld[r] = gl;
      a0 += loss;
      a1 += ce;
      a2 += ldr;
    }
  }
  if (kind < 0) return;
  if (lane == 0) {
    red[wv][0] = a0;
    red[wv][1] = a1;
    red[wv][2] = a2;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    float v = 0.f;
    if (threadIdx.x < 3)
      for (int q = 0; q < 4; ++q) v += red[q][threadIdx.x];
    partials[blockIdx.x * 4 + threadIdx.x] = v;
  }
}

// Back through one coupling update, one wave per row: undo the flip /
// permutation (g_pre[fq[j]] = g_out[j]), then with e = e^{s}:
//   G_s = g_pre_T x_T e + gld,  G_t = g_pre_T,  g_in_T = g_pre_T e,
//   g_in_C = g_pre_C (the conditioners' share is added by the first Linear's
//   back-prop), plus the caller's gradient of the previous layer's output.
// strict: torch autograd's rules for the op sequence of k_wfwd_update over
// every feature (b_1 = 1 - mask):  g_v = g b_1, G_t = g_v,
//   G_s = (g_v x) e + gld b_1,  g_in = g mask + g_v e  (0 * inf = NaN kept).
// kRU rows per wave with every load of the group issued first (as k_wfwd_update).
template <int kNJ>
__global__ __launch_bounds__(256) void k_wbwd_update(
    const float* __restrict__ gout, float* __restrict__ gin, const float* __restrict__ X,
    const float* __restrict__ Os, const float* __restrict__ gld, float* __restrict__ Gs,
    float* __restrict__ Gt, const float* __restrict__ gprev, const int32_t* __restrict__ fqg,
    int64_t B, Geo g) {
  __shared__ int32_t sq[CNF_MAX_DIM];
  const int32_t* fq = stage_table(sq, fqg, g.D);
  const int lane = threadIdx.x & 63;
  const int D = g.D, DT = g.DT, Op = g.Op;
  int ii[kNJ];
#pragma unroll
  for (int q = 0; q < kNJ; ++q) ii[q] = lane + 64 * q < D ? fq[lane + 64 * q] : 0;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * kRU; r0 < B; r0 += nw * kRU) {
    float vo[kRU][kNJ], xt[kRU][kNJ], sv[kRU][kNJ], gp[kRU][kNJ], gl[kRU];
#pragma unroll
    for (int u = 0; u < kRU; ++u) {
      const int64_t r = r0 + u < B ? r0 + u : B - 1;  // past-the-end rows: loads only
      gl[u] = gld[r];
#pragma unroll
      for (int q = 0; q < kNJ; ++q) {
        const int j = lane + 64 * q, i = ii[q];
        vo[u][q] = xt[u][q] = sv[u][q] = gp[u][q] = 0.f;
        if (j < D) {
          vo[u][q] = gout[r * D + j];
          if (i < DT || g.strict) {
            xt[u][q] = X[r * g.Dp + g.col(i)];
            if (Os) sv[u][q] = Os[r * Op + i];
          }
          if (gprev) gp[u][q] = gprev[r * D + i];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < kRU; ++u) {
      const int64_t r = r0 + u;
      if (r >= B) break;
#pragma unroll
      for (int q = 0; q < kNJ; ++q) {
        const int j = lane + 64 * q, i = ii[q];
        if (j >= D) continue;
        const float v = vo[u][q];
        float gi = v;
        if (g.strict) {
          const float b1 = i < DT ? 1.f : 0.f;
          const float e = Os ? expf(sv[u][q]) : 1.f;
          const float gv = __fmul_rn(v, b1);
          if (Gs) Gs[r * Op + i] = __fadd_rn(__fmul_rn(__fmul_rn(gv, xt[u][q]), e), __fmul_rn(gl[u], b1));
          if (Gt) Gt[r * Op + i] = gv;
          gi = __fadd_rn(__fmul_rn(v, 1.f - b1), __fmul_rn(gv, e));
        } else if (i < DT) {
          const float e = Os ? expf(sv[u][q]) : 1.f;
          if (Gs) Gs[r * Op + i] = __fadd_rn(__fmul_rn(__fmul_rn(v, xt[u][q]), e), gl[u]);
          if (Gt) Gt[r * Op + i] = v;
          gi = __fmul_rn(v, e);
        }
        if (gprev) gi += gp[u][q];
        gin[r * D + i] = gi;
      }
      for (int i = (g.strict ? D : DT) + lane; i < Op; i += 64) {
        if (Gs) Gs[r * Op + i] = 0.f;
        if (Gt) Gt[r * Op + i] = 0.f;
      }
    }
  }
}

// ---- the inverse transform's reverse mode (wvjp_inv_run) ----

// z natural -> stash layout of the first inverse step's gathered input
// z'[j] = z[iq[j]] (flip and rev_perm undone, flows/flows.py:115-117).
// strict: the C part is the reference's whole x_b = mask * z' (0 * z'_T at the
// mask's zero columns: NaN where z'_T is not finite), raw z'_T in the T part.
__global__ __launch_bounds__(256) void k_winv_stash(const float* __restrict__ z,
                                                    const int32_t* __restrict__ iqg,
                                                    float* __restrict__ xs, int64_t B, Geo g) {
  __shared__ int32_t sq[CNF_MAX_DIM];
  const int32_t* iq = stage_table(sq, iqg, g.D);
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < B; r += nw) {
    for (int j = lane; j < g.D; j += 64) {
      const float v = z[r * g.D + iq[j]];
      xs[r * g.Dp + g.col(j)] = v;
      if (g.strict && j < g.DT) xs[r * g.Dp + j] = 0.f * v;
    }
    for (int c = g.ones() + lane; c < g.Cp; c += 64) xs[r * g.Dp + c] = c == g.ones() ? 1.f : 0.f;
    for (int c = g.Cp + g.DT + lane; c < g.Dp; c += 64) xs[r * g.Dp + c] = 0.f;
  }
}

// One inverse step (flows/flows.py:118-126): x_T = (z'_T - t) e^{-s}, x_C = z'_C;
// written straight into the next step's gathered stash slot (x[iq_next[j]]).
// strict: the reference's own op sequence over every feature (b_1 = 1 - mask),
//   x = x_b + (b_1 (z' - t)) e^{-s},  one rounding per op, so 0 * inf = NaN
// at masked positions as in torch; the next slot's C part gets x_b again.
__global__ __launch_bounds__(256) void k_winv_fwd_update(const float* __restrict__ X,
                                                         float* __restrict__ Xn,
                                                         const float* __restrict__ Os,
                                                         const float* __restrict__ Ot,
                                                         const int32_t* __restrict__ iqg,
                                                         int64_t B, Geo g) {
  __shared__ int32_t sq[CNF_MAX_DIM];
  const int32_t* iqn = stage_table(sq, iqg, g.D);
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < B; r += nw) {
    const float* xr = X + r * g.Dp;
    float* zr = Xn + r * g.Dp;
    for (int j = lane; j < g.D; j += 64) {
      const int i = iqn[j];  // next step's z'[j] = this step's x[i]
      float v = xr[g.col(i)];
      if (g.strict) {
        const float b1 = i < g.DT ? 1.f : 0.f;
        const float sv = Os ? Os[r * g.Op + i] : 0.f;
        const float tv = Ot ? Ot[r * g.Op + i] : 0.f;
        const float c = __fmul_rn(b1, __fsub_rn(v, tv));
        v = __fadd_rn(__fmul_rn(1.f - b1, v), __fmul_rn(c, expf(-sv)));
        if (j < g.DT) zr[j] = 0.f * v;  // the next step's x_b (mask 0 here)
      } else if (i < g.DT) {
        const float sv = Os ? Os[r * g.Op + i] : 0.f;
        const float tv = Ot ? Ot[r * g.Op + i] : 0.f;
        v = __fmul_rn(__fsub_rn(v, tv), expf(-sv));
      }
      zr[g.col(j)] = v;
    }
    for (int c = g.ones() + lane; c < g.Cp; c += 64) zr[c] = c == g.ones() ? 1.f : 0.f;
    for (int c = g.Cp + g.DT + lane; c < g.Dp; c += 64) zr[c] = 0.f;
  }
}

// Back through one inverse step's coupling: g (natural, this step's output) ->
// tmp (gathered order z'), G_s / G_t for the conditioners.
// strict: torch autograd's rules for the op sequence of k_winv_fwd_update
// (c = b_1 (z' - t), x = x_b + c e, e = e^{-s}, ld -= sum b_1 s):
//   g_c = g e,  G_s = -((g c) e) - gld b_1,  G_t = -(g_c b_1),
//   g_{z'} = g_c b_1 + mask g   (the conditioners' share, mask-weighted, is
//   added by the first Linear's back-prop: kEpiAdd with zlt = DT).
__global__ __launch_bounds__(256) void k_winv_bwd_update(
    const float* __restrict__ gout, float* __restrict__ tmp, const float* __restrict__ X,
    const float* __restrict__ Os, const float* __restrict__ Ot, const float* __restrict__ gld,
    float* __restrict__ Gs, float* __restrict__ Gt, int64_t B, Geo g) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int D = g.D, DT = g.DT, Op = g.Op;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < B; r += nw) {
    const float gl = gld[r];
    for (int j = lane; j < D; j += 64) {
      const float v = gout[r * D + j];
      float gz = v;
      if (g.strict) {
        const float b1 = j < DT ? 1.f : 0.f;
        const float s = Os ? Os[r * Op + j] : 0.f;
        const float t = Ot ? Ot[r * Op + j] : 0.f;
        const float e = expf(-s);
        const float c = __fmul_rn(b1, __fsub_rn(X[r * g.Dp + g.col(j)], t));
        const float gc = __fmul_rn(v, e);
        const float ga = __fmul_rn(gc, b1);
        if (Gs) Gs[r * Op + j] = __fsub_rn(-__fmul_rn(__fmul_rn(v, c), e), __fmul_rn(gl, b1));
        if (Gt) Gt[r * Op + j] = -ga;
        gz = __fadd_rn(ga, __fmul_rn(1.f - b1, v));
      } else if (j < DT) {
        const float s = Os ? Os[r * Op + j] : 0.f;
        const float t = Ot ? Ot[r * Op + j] : 0.f;
        const float e = expf(-s);
        const float xT = __fmul_rn(__fsub_rn(X[r * g.Dp + g.Cp + j], t), e);
        gz = __fmul_rn(v, e);
        if (Gs) Gs[r * Op + j] = __fsub_rn(-__fmul_rn(v, xT), gl);
        if (Gt) Gt[r * Op + j] = -gz;
      }
      tmp[r * D + j] = gz;
    }
    for (int i = (g.strict ? D : DT) + lane; i < Op; i += 64) {
      if (Gs) Gs[r * Op + i] = 0.f;
      if (Gt) Gt[r * Op + i] = 0.f;
    }
  }
}

// g_{z_in}[iq[j]] = tmp[j] (+ the caller's gradient of that output); skip: no
// destination wanted (dz == NULL on the last step)
__global__ __launch_bounds__(256) void k_winv_scatter(const float* __restrict__ tmp,
                                                      float* __restrict__ out,
                                                      const float* __restrict__ gprev,
                                                      const int32_t* __restrict__ iqg, int64_t B,
                                                      int D, int skip) {
  if (skip) return;
  __shared__ int32_t sq[CNF_MAX_DIM];
  const int32_t* iq = stage_table(sq, iqg, D);
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < B; r += nw) {
    for (int j = lane; j < D; j += 64) {
      const int i = iq[j];
      float v = tmp[r * D + j];
      if (gprev) v += gprev[r * D + i];
      out[r * D + i] = v;
    }
  }
}

inline int64_t al64(int64_t floats) { return (floats + 63) / 64 * 64; }

// the instantiation whose column slots per lane cover D
template <class F>
F pick_nj(int D, F f1, F f2, F f3, F f4) {
  return D <= 64 ? f1 : (D <= 128 ? f2 : (D <= 192 ? f3 : f4));
}

// strict: the first Linear sees all D inputs, the last writes all D outputs
int lin_out(const Shape& s, int k) {
  return k == s.n_lin - 1 ? (s.strict ? s.D : s.DT) : s.units[k + 1];
}
int lin_in(const Shape& s, int k) { return k == 0 ? (s.strict ? s.D : s.DC) : s.units[k]; }
int hp(const Shape& s, int k) { return r8(s.units[k + 1] + 1); }  // H_k: units + ones
int gp(const Shape& s, int k) { return r8(lin_out(s, k)); }       // G_k

Geo geo(const Shape& s) {
  Geo g;
  g.D = s.D;
  g.DT = s.DT;
  g.DC = s.DC;
  g.strict = s.strict ? 1 : 0;
  g.Cp = r8((s.strict ? s.D : s.DC) + 1);
  g.DTp = r8(s.DT);
  g.Dp = g.Cp + g.DTp;
  g.Op = r8(s.strict ? s.D : s.DT);
  return g;
}

// Workspace plan (float offsets), shared by the size query and the run.
struct Plan {
  int64_t stash, ld, gld, g0, g1, seed, part;
  int64_t H[2][kMaxLin], O[2], G[2][kMaxLin];
  int64_t act_stride;  // floats between layers' H / O (keep_acts), else 0
  bool keep_acts;      // every layer's conditioner activations kept from the forward sweep
  int64_t total;
  int64_t nkb, rows_kb, nseed;
};

// Keeping every layer's conditioner activations (instead of recomputing them
// in the backward sweep) costs no extra HBM traffic -- the forward sweep
// writes them anyway -- only workspace; kept up to this many bytes.
constexpr double kKeepActsBytes = 8.0 * (1 << 30);

Plan make_plan(const Shape& s, int64_t B) {
  Plan p{};
  const int64_t Bn = B > 0 ? B : 1;
  const Geo g = geo(s);
  int64_t off = 0;
  auto take = [&](int64_t n) {
    const int64_t o = off;
    off += al64(n);
    return o;
  };
  p.stash = take((int64_t)(s.L + 1) * Bn * g.Dp);
  p.ld = take(Bn);
  p.gld = take(Bn);
  p.g0 = take(Bn * s.D);
  p.g1 = take(Bn * s.D);
  int64_t acts = 0;  // floats of one layer's H / O, all nets
  for (int n = 0; n < s.nets; ++n) {
    for (int k = 0; k + 1 < s.n_lin; ++k) acts += al64(Bn * hp(s, k));
    acts += al64(Bn * g.Op);
  }
  p.keep_acts = s.L > 1 && (double)acts * s.L * 4 <= kKeepActsBytes;
  p.act_stride = p.keep_acts ? acts : 0;
  const int64_t act0 = take(acts * (p.keep_acts ? s.L : 1));
  int64_t a = act0;
  for (int n = 0; n < s.nets; ++n) {
    for (int k = 0; k + 1 < s.n_lin; ++k) {
      p.H[n][k] = a;
      a += al64(Bn * hp(s, k));
    }
    p.O[n] = a;
    a += al64(Bn * g.Op);
  }
  for (int n = 0; n < s.nets; ++n)
    for (int k = 0; k < s.n_lin; ++k) p.G[n][k] = take(Bn * gp(s, k));
  p.nseed = std::min<int64_t>(4096, (Bn + 15) / 16);  // one wave per row: 16 rows per wave at 2^18
  p.seed = take(p.nseed * 4);
  int64_t rows = (Bn + 255) / 256;
  rows = std::max<int64_t>(256, (rows + 31) / 32 * 32);
  p.rows_kb = rows;
  p.nkb = (Bn + rows - 1) / rows;
  p.part = take(p.nkb * al64(s.layer_floats));
  p.total = off;
  return p;
}

int64_t lin_off(const Shape& s, int k) {
  int64_t o = 0;
  for (int i = 0; i < k; ++i) o += (int64_t)s.units[i + 1] * s.units[i] + s.units[i + 1];
  return o;
}

int check_launch() {
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    set_hip_error(err);
    return CNF_ERR_HIP;
  }
  return CNF_OK;
}

int gemm_nc(int cols) { return std::min(kBN / 32, (cols + 31) / 32); }

size_t gemm_lds(int cols, int K, bool pair) {
  return (size_t)((K + 7) & ~7) * (32 * gemm_nc(cols) + 8) * 4 * (pair ? 2 : 1);
}

template <int NC>
void launch_nc(bool bt, int epi, bool pair, dim3 grid, size_t lds, hipStream_t st,
               const GemmArgs& ga) {
  if (bt && epi == kEpiBias)
    hipLaunchKernelGGL((k_wgemm<true, kEpiBias, false, NC>), grid, dim3(256), lds, st, ga);
  else if (bt && epi == kEpiBiasRelu)
    hipLaunchKernelGGL((k_wgemm<true, kEpiBiasRelu, false, NC>), grid, dim3(256), lds, st, ga);
  else if (!bt && epi == kEpiMask)
    hipLaunchKernelGGL((k_wgemm<false, kEpiMask, false, NC>), grid, dim3(256), lds, st, ga);
  else if (!bt && epi == kEpiAdd && pair)
    hipLaunchKernelGGL((k_wgemm<false, kEpiAdd, true, NC>), grid, dim3(256), lds, st, ga);
  else
    hipLaunchKernelGGL((k_wgemm<false, kEpiAdd, false, NC>), grid, dim3(256), lds, st, ga);
}

// One GEMM launch over B rows; cols = columns written (N plus pad).
void gemm(GemmArgs ga, int64_t B, int cols, int K, int nz, bool bt, int epi, bool pair,
          hipStream_t st) {
  const unsigned ny = (unsigned)((cols + kBN - 1) / kBN);
  const size_t lds = gemm_lds(cols, K, pair);
  const int per_cu = (int)std::max<size_t>(1, std::min<size_t>(4, 160 * 1024 / lds));
  const int64_t want = std::max<int64_t>(1, (int64_t)256 * per_cu / (ny * nz));
  const int64_t nx = (std::min<int64_t>(want, ((B + 31) / 32 + 3) / 4) + 7) / 8 * 8;
  const dim3 grid((unsigned)(nx * ny), 1, (unsigned)nz);
  ga.ny = (int)ny;
  switch (gemm_nc(cols)) {
    case 1: launch_nc<1>(bt, epi, pair, grid, lds, st, ga); break;
    case 2: launch_nc<2>(bt, epi, pair, grid, lds, st, ga); break;
    default: launch_nc<2>(bt, epi, pair, grid, lds, st, ga); break;
  }
}

}  // namespace

// Every Linear's weight slice (K x 32*NC floats, both nets for the paired
// launch) must fit one CU's LDS: widths up to ~290 (CNF_MAX_WIDTH 512 shapes
// beyond that keep the torch fallback).
bool wvjp_ok(const Shape& s) {
  if (s.strict && (s.alt_mask || s.s_tanh)) return false;
  constexpr size_t kLds = 160 * 1024;
  // column counts as the launches use them: a strict stack's last Linear
  // writes all D columns, and its first-Linear back-prop produces all D
  // input columns (x_b = mask * x), not DT / DC
  for (int k = 0; k < s.n_lin; ++k) {
    const int cols = k == s.n_lin - 1 ? lin_out(s, k) : hp(s, k);
    if (gemm_lds(cols, lin_in(s, k), false) > kLds) return false;               // forward
    if (k > 0 && gemm_lds(gp(s, k - 1), lin_out(s, k), false) > kLds) return false;  // back-prop
  }
  return gemm_lds(s.strict ? s.D : s.DC, lin_out(s, 0), s.nets == 2) <= kLds;
}

namespace {

// ---- the fused training sweeps (cnf_wide16.hip: k_wtrain16_fwd / _bwd) ----
// For the stacks k_wide16 serves, the layer-at-a-time GEMMs and update
// kernels above give way to one forward launch (every layer, activations in
// registers, a per-row tape written on the way) and one reverse launch per
// layer; k_wseed and the weight-gradient launch (k_wdw16 on the slot-order
// operands) stay.  Workspace: the tape of every layer (L x B x RW floats:
// cfg4 at 2^18 rows 8.1 GB), the final output in the stash layout the seed
// reads, ld / gld, two natural-order gradients, one layer's conditioner
// gradients (B x GW), the seed and dW partials.
struct Plan16 {
  int64_t tape, tbits, zst, ld, gld, g0, gbuf, seed, part, total, nkb, rows_kb, nseed;
};
constexpr double kTapeMaxBytes = 96.0 * (1ull << 30);  // beyond: the layer-at-a-time path
#ifndef CNF_WDWG_NKB
#define CNF_WDWG_NKB 256
#endif

bool plan16(const Shape& s, int64_t B, WTrain16Layout* lay, Plan16* p) {
  if (!wide16_train_ok(s) || wide16_train_layout(s, lay) != CNF_OK) return false;
  const int64_t Bn = B > 0 ? B : 1;
  const int64_t Bp = wide16_blocks(Bn) * 32;  // whole 32-row blocks (wave-tiled arrays)
  if ((double)s.L * Bp * (lay->RW + lay->GW) * 4 > kTapeMaxBytes) return false;
  const Geo g = geo(s);
  int64_t off = 0;
  auto take = [&](int64_t n) {
    const int64_t o = off;
    off += al64(n);
    return o;
  };
  p->tape = take((int64_t)s.L * Bp * lay->RW);
  p->tbits = take((int64_t)s.L * wide16_tbits_words(Bn));
  p->zst = take(Bn * g.Dp);
  p->ld = take(Bn);
  p->gld = take(Bn);
  p->g0 = take(Bn * s.D);
  p->gbuf = take((int64_t)s.L * Bp * lay->GW);
  p->nseed = std::min<int64_t>(4096, (Bn + 15) / 16);  // k_wseed's blocks (generic seeds)
  p->seed = take(std::max<int64_t>(p->nseed, wide16_blocks(Bn)) * 4);  // or one record per wave
  // k_wdw16g's row blocks: CNF_WDWG_NKB of them (each one record of dW
  // partials that the fixed-order reduction reads back).  At cfg4 (2^18 rows)
  // 256 measured 255 us per layer; 128 / 171 / 512 blocks 300 / 293 / 278 us
  // (fewer blocks: a ragged last round of the 2-per-CU grid; more: partials)
  int64_t rows = (Bn + CNF_WDWG_NKB - 1) / CNF_WDWG_NKB;
  rows = std::max<int64_t>(256, (rows + 31) / 32 * 32);
  p->rows_kb = rows;
  p->nkb = (Bn + rows - 1) / rows;
  p->part = take(p->nkb * al64(s.layer_floats));
  p->total = off;
  return true;
}

int wvjp16_run(const Shape& s, const WTrain16Layout& lay, const Plan16& p, const void* prepared,
               const float* x, const int64_t* y, const float* gz, const float* gz_all,
               const float* gld_in, int kind, float det, float grad_scale, float* loss_terms,
               float* grads, float* dx, int64_t B, float* W, hipStream_t st) {
  const Geo geom = geo(s);
  const int D = s.D, L = s.L, NL = s.n_lin;
  float* ld = W + p.ld;
  float* gld = W + p.gld;
  float* tape = W + p.tape;
  uint32_t* tbits = reinterpret_cast<uint32_t*>(W + p.tbits);
  float* g[1] = {W + p.g0};
  if (kind >= 0) {  // the loss seed rides the forward sweep's epilogue
    const WSeed16 sd{y, g[0], gld, W + p.seed, det, grad_scale, kind};
    int r = wide16_train_forward(s, prepared, x, W + p.zst, geom.Cp, geom.Dp, ld, tape, tbits, B,
                                 &sd, st);
    if (r != CNF_OK) return r;
    reduce_partials(W + p.seed, (int)wide16_blocks(B), 4, 0, nullptr, loss_terms, st);
  } else {
    int r = wide16_train_forward(s, prepared, x, W + p.zst, geom.Cp, geom.Dp, ld, tape, tbits, B,
                                 nullptr, st);
    if (r != CNF_OK) return r;
    hipLaunchKernelGGL(k_wseed, dim3((unsigned)p.nseed), dim3(256), 0, st, W + p.zst, ld, y, kind,
                       det, grad_scale, gz, gz_all ? gz_all + (int64_t)(L - 1) * B * D : nullptr,
                       gld_in, g[0], gld, W + p.seed, B, geom);
  }
  const int64_t PL = s.layer_floats, PS = al64(PL);
  float* part = W + p.part;
  if (PL > 0 && hipMemsetAsync(part, 0, (size_t)p.nkb * PS * 4, st) != hipSuccess)
    return check_launch();
  int r = wide16_train_backward(s, prepared, g[0], gz_all, dx, gld, tape, tbits, W + p.gbuf, B, st);
  if (r != CNF_OK) return r;
  const int64_t Bp = wide16_blocks(B) * 32;
  for (int l = L - 1; l >= 0; --l) {
    const float* tl = tape + (int64_t)l * Bp * lay.RW;
    const float* gl = W + p.gbuf + (int64_t)l * Bp * lay.GW;
    DwArgs da{};
    da.partials = part;
    da.M = B;
    da.rows = p.rows_kb;
    da.PS = PS;
    int jobs = 0, max_subs = 1;
    for (int n = 0; n < s.nets; ++n)
      for (int k = 0; k < NL; ++k) {
        DwJob& j = da.job[jobs++];
        const bool last = k == NL - 1;
        // wave-tiled parts: a part starting at column c begins (c / 16) * 512
        // floats into each 32-row block
        j.G = gl + (int64_t)(last ? lay.glast[n] : lay.gpre[n][k + 1]) / 16 * 512;
        j.ldg = lay.GW;
        j.gcl = (last ? lay.ts : lay.gpw[k + 1]) - 1;
        j.H = tl + (int64_t)(k == 0 ? lay.xc : lay.h[n][k]) / 16 * 512;
        j.ldh = lay.RW;
        j.hcl = (k == 0 ? lay.cw : lay.hw[k]) - 1;
        j.N = last ? s.DT : s.units[k + 1];
        j.K = k == 0 ? s.DC : s.units[k];
        j.slot = 1;
        j.cstep = 1;
        j.rrev = 0;
        j.nfull = s.units[k + 1];
        j.woff = n * s.net_floats + lin_off(s, k) + (k == 0 ? s.DT : 0);
        j.wld = s.units[k];
        j.boff = n * s.net_floats + lin_off(s, k) + (int64_t)s.units[k + 1] * s.units[k];
        j.tiles_c = (j.K + 1 + 31) / 32;
        const int ncg = ((j.K + 1 + 15) / 16 + kDw16CT - 1) / kDw16CT;
        max_subs = std::max(max_subs, ((j.N + 127) / 128) * ncg);
      }
    int maxtpc = 0;
    bool gok = CNF_WDW16G;
    for (int q = 0; q < jobs; ++q) {
      const int ng = (da.job[q].gcl >> 4) + 1, nh = (da.job[q].hcl >> 4) + 1;
      gok = gok && wdwg_class_ok(ng, nh);
      maxtpc = std::max(maxtpc, ng + nh);
    }
    if (gok) {  // whole 32-row blocks (padding rows carry zero G)
      da.M = Bp;
      hipLaunchKernelGGL(k_wdw16g, dim3((unsigned)p.nkb, (unsigned)jobs), dim3(256),
                         (size_t)2 * maxtpc * 2048, st, da);
    } else {
      hipLaunchKernelGGL(k_wdw16, dim3((unsigned)p.nkb, (unsigned)jobs, (unsigned)max_subs),
                         dim3(256), 0, st, da);
    }
    reduce_partials(part, (int)p.nkb, (int)PS, (int)PL, grads + (int64_t)l * PL, nullptr, st);
  }
  return check_launch();
}

}  // namespace

int wvjp_workspace(const Shape& s, int64_t B, size_t* bytes) {
  if (!wvjp_ok(s)) return CNF_ERR_UNSUPPORTED;
  WTrain16Layout lay;
  Plan16 p16;
  *bytes = (size_t)(plan16(s, B, &lay, &p16) ? p16.total : make_plan(s, B).total) * 4;
  return CNF_OK;
}

// the inverse transform's reverse mode always runs layer at a time
int wvjp_inv_workspace(const Shape& s, int64_t B, size_t* bytes) {
  if (!wvjp_ok(s)) return CNF_ERR_UNSUPPORTED;
  *bytes = (size_t)make_plan(s, B).total * 4;
  return CNF_OK;
}

namespace {

// Host side of one layer-at-a-time sweep: workspace views and the per-layer
// launch sequences shared by the forward transform's reverse mode (wvjp_run)
// and the inverse transform's (wvjp_inv_run).  A "slot" indexes the stashed
// inputs / kept activations in sweep order, a "layer" the parameters.
struct Runner {
  const Shape& s;
  const Plan& p;
  float* W;
  const float* plain;
  Geo geom;
  int64_t B;
  hipStream_t st;
  int D, DT, DC, NL, L;
  int64_t PL, PS, Dp;
  unsigned wave_blocks;
  int dw_calls = 0;

  Runner(const Shape& s_, const Plan& p_, void* ws, const void* prepared, int64_t B_,
         hipStream_t st_)
      : s(s_), p(p_), W(static_cast<float*>(ws)),
        plain(reinterpret_cast<const float*>(static_cast<const char*>(prepared) + idx_bytes(s_)) +
              s_.plain_region),
        geom(geo(s_)), B(B_), st(st_), D(s_.D), DT(s_.DT), DC(s_.DC), NL(s_.n_lin), L(s_.L),
        PL(s_.layer_floats), PS(al64(s_.layer_floats)), Dp(geo(s_).Dp),
        wave_blocks((unsigned)std::min<int64_t>((B_ + 3) / 4, 16384)) {}

  float* Xs(int slot) const { return W + p.stash + (int64_t)slot * B * Dp; }
  float* Hb(int slot, int n, int k) const {
    return W + p.H[n][k] + (int64_t)slot * p.act_stride;
  }
  float* Ob(int slot, int n) const { return W + p.O[n] + (int64_t)slot * p.act_stride; }
  const float* Os(int slot) const { return s.scale ? Ob(slot, 0) : nullptr; }
  const float* Ot(int slot) const { return s.shift ? Ob(slot, s.scale) : nullptr; }
  float* Gk(int n, int k) const { return W + p.G[n][k]; }
  const float* wptr(int layer, int n, int k) const {
    return plain + layer * PL + n * s.net_floats + lin_off(s, k);
  }
  const float* bptr(int layer, int n, int k) const {
    return wptr(layer, n, k) + (int64_t)s.units[k + 1] * s.units[k];
  }
  int act(int n) const { return (s.s_tanh && s.scale && n == 0) ? 2 : 1; }

  // both conditioners of `layer` on the conditioning half of slot `slot`
  void nets_forward(int slot, int layer) const {
    for (int k = 0; k < NL; ++k) {
      GemmArgs ga{};
      ga.M = B;
      const bool last = k == NL - 1;
      for (int n = 0; n < s.nets; ++n) {
        GemmJob& j = ga.job[n];
        j.A = k == 0 ? Xs(slot) : Hb(slot, n, k - 1);
        j.lda = k == 0 ? Dp : hp(s, k - 1);
        j.K = lin_in(s, k);
        j.Bw = wptr(layer, n, k) + (k == 0 && !s.strict ? DT : 0);
        j.ldb = s.units[k];
        j.N = lin_out(s, k);
        j.bias = bptr(layer, n, k);
        j.C = last ? Ob(slot, n) : Hb(slot, n, k);
        j.ldc = last ? geom.Op : hp(s, k);
        j.ldw = last ? j.N : hp(s, k);
        j.ones = !last;
        j.act = act(n);
      }
      gemm(ga, B, ga.job[0].ldw, lin_in(s, k), s.nets, true, last ? kEpiBias : kEpiBiasRelu,
           false, st);
    }
  }

  // back through both conditioners from their output gradients Gk(n, NL-1):
  // G_{k-1} = (G_k W_k) * act'(H_{k-1}), then gin[:, DT:] += sum_n G_0 W_0[:, DT:]
  void nets_backward(int slot, int layer, float* gin) const {
    for (int k = NL - 1; k >= 1; --k) {
      GemmArgs ga{};
      ga.M = B;
      for (int n = 0; n < s.nets; ++n) {
        GemmJob& j = ga.job[n];
        j.A = Gk(n, k);
        j.lda = gp(s, k);
        j.K = lin_out(s, k);
        j.Bw = wptr(layer, n, k);
        j.ldb = s.units[k];
        j.N = s.units[k];
        j.C = Gk(n, k - 1);
        j.ldc = gp(s, k - 1);
        j.ldw = gp(s, k - 1);
        j.mask = Hb(slot, n, k - 1);
        j.ldm = hp(s, k - 1);
        j.act = act(n);
      }
      gemm(ga, B, gp(s, k - 1), lin_out(s, k), s.nets, false, kEpiMask, false, st);
    }
    GemmArgs ga{};
    ga.M = B;
    GemmJob& j = ga.job[0];
    j.A = Gk(0, 0);
    j.lda = gp(s, 0);
    j.K = lin_out(s, 0);
    const int c0 = s.strict ? 0 : DT;  // strict: every input column (x_b = mask * x)
    j.Bw = wptr(layer, 0, 0) + c0;
    j.ldb = D;
    if (s.nets == 2) {
      j.A2 = Gk(1, 0);
      j.lda2 = j.lda;
      j.Bw2 = wptr(layer, 1, 0) + c0;
      j.ldb2 = D;
    }
    j.N = s.strict ? D : DC;
    j.C = gin + c0;
    j.zlt = s.strict ? DT : 0;
    j.ldc = D;
    j.ldw = j.N;
    gemm(ga, B, j.N, j.K, 1, false, kEpiAdd, s.nets == 2, st);
  }

  // weight / bias gradients of every Linear of both nets (one launch) into the
  // per-row-block partials, then their fixed-order sum into grads_layer
  int weight_grads(int slot, int layer, float* grads_layer) {
    float* part = W + p.part;
    // the records are reused across layers: positions a layer never writes
    // (masked columns / rows) keep the first memset's zeros, except that under
    // the legacy alternate mask odd and even layers mask different positions
    if (s.alt_mask && dw_calls > 0 &&
        hipMemsetAsync(part, 0, (size_t)p.nkb * PS * 4, st) != hipSuccess)
      return check_launch();
    ++dw_calls;
    DwArgs da{};
    da.partials = part;
    da.M = B;
    da.rows = p.rows_kb;
    da.PS = PS;
    int jobs = 0, max_subs = 1;
    for (int n = 0; n < s.nets; ++n) {
      for (int k = 0; k < NL; ++k) {
        DwJob& j = da.job[jobs++];
        j.G = Gk(n, k);
        j.ldg = gp(s, k);
        j.H = k == 0 ? Xs(slot) : Hb(slot, n, k - 1);
        j.ldh = k == 0 ? Dp : hp(s, k - 1);
        j.N = lin_out(s, k);
        j.K = lin_in(s, k);
        // legacy alternate mask: an odd layer's kernel weights are its
        // parameters with the first Linear's columns and the last Linear's
        // rows reversed (cnf_tile.hip prepare); map the gradients back
        const bool rev = s.alt_mask && (layer & 1);
        const bool rin = rev && k == 0, rout = rev && k == NL - 1;
        j.cstep = rin ? -1 : 1;
        j.rrev = rout;
        j.nfull = s.units[k + 1];
        j.woff = n * s.net_floats + lin_off(s, k) +
                 (k == 0 && !s.strict ? (rin ? D - 1 - DT : DT) : 0);
        j.wld = s.units[k];
        j.boff = n * s.net_floats + lin_off(s, k) + (int64_t)s.units[k + 1] * s.units[k];
        j.tiles_c = (j.K + 1 + 31) / 32;
        j.gcl = j.N - 1;
        j.hcl = (int)j.ldh - 1;
        j.slot = 0;
#if CNF_WDW16
        const int ncg = ((j.K + 1 + 15) / 16 + kDw16CT - 1) / kDw16CT;
#else
        const int ncg = (j.tiles_c + kDwCT - 1) / kDwCT;
#endif
        max_subs = std::max(max_subs, ((j.N + 127) / 128) * ncg);
      }
    }
#if CNF_WDW16
    hipLaunchKernelGGL(k_wdw16,
#else
    hipLaunchKernelGGL(k_wdw,
#endif
                       dim3((unsigned)p.nkb, (unsigned)jobs, (unsigned)max_subs), dim3(256), 0, st,
                       da);
    reduce_partials(part, (int)p.nkb, (int)PS, (int)PL, grads_layer, nullptr, st);
    return CNF_OK;
  }
};

int empty_batch(const Shape& s, float* grads, float* loss_terms, hipStream_t st) {
  const int64_t P = s.layer_floats * s.L;
  if (P > 0 && hipMemsetAsync(grads, 0, (size_t)P * 4, st) != hipSuccess) return check_launch();
  if (loss_terms && hipMemsetAsync(loss_terms, 0, 3 * 4, st) != hipSuccess) return check_launch();
  return check_launch();
}

}  // namespace

int wvjp_run(const Shape& s, const void* prepared, const float* x, const int64_t* y,
             const float* gz, const float* gz_all, const float* gld_in, int kind, float det,
             float grad_scale, float* loss_terms, float* grads, float* dx, int64_t B, void* ws,
             size_t ws_bytes, hipStream_t st) {
  if (!wvjp_ok(s)) return CNF_ERR_UNSUPPORTED;
  {
    WTrain16Layout lay;
    Plan16 p16;
    if (plan16(s, B, &lay, &p16)) {
      if (!ws || ws_bytes < (size_t)p16.total * 4) return CNF_ERR_NULL;
      if (B == 0) return empty_batch(s, grads, loss_terms, st);
      return wvjp16_run(s, lay, p16, prepared, x, y, gz, gz_all, gld_in, kind, det, grad_scale,
                        loss_terms, grads, dx, B, static_cast<float*>(ws), st);
    }
  }
  const Plan p = make_plan(s, B);
  if (!ws || ws_bytes < (size_t)p.total * 4) return CNF_ERR_NULL;
  if (B == 0) return empty_batch(s, grads, loss_terms, st);
  Runner R(s, p, ws, prepared, B, st);
  const int32_t* fq = reinterpret_cast<const int32_t*>(prepared);
  const int D = s.D, NL = s.n_lin, L = s.L;
  float* W = R.W;
  float* ld = W + p.ld;
  float* gld = W + p.gld;

  // ---- forward sweep: slot l = input of layer l ----
  hipLaunchKernelGGL(k_wstash, dim3(R.wave_blocks), dim3(256), 0, st, x, R.Xs(0), B, R.geom);
  for (int l = 0; l < L; ++l) {
    if (s.nets) R.nets_forward(l, l);
    hipLaunchKernelGGL(pick_nj(D, k_wfwd_update<1>, k_wfwd_update<2>, k_wfwd_update<3>,
                               k_wfwd_update<4>),
                       dim3(R.wave_blocks), dim3(256), 0, st, R.Xs(l), R.Xs(l + 1),
                       ld, R.Os(l), R.Ot(l), fq + l * D, B, R.geom, l == 0);
  }
  // ---- seed ----
  float* g[2] = {W + p.g0, W + p.g1};
  int cur = 0;
  hipLaunchKernelGGL(k_wseed, dim3((unsigned)p.nseed), dim3(256), 0, st, R.Xs(L), ld, y, kind, det,
                     grad_scale, gz, gz_all ? gz_all + (int64_t)(L - 1) * B * D : nullptr, gld_in,
                     g[0], gld, W + p.seed, B, R.geom);
  if (kind >= 0) reduce_partials(W + p.seed, (int)p.nseed, 4, 0, nullptr, loss_terms, st);
  if (R.PL > 0 && hipMemsetAsync(W + p.part, 0, (size_t)p.nkb * R.PS * 4, st) != hipSuccess)
    return check_launch();

  // ---- backward sweep ----
  for (int l = L - 1; l >= 0; --l) {
    if (s.nets && !p.keep_acts) R.nets_forward(l, l);  // recompute, or the kept activations
    float* gin = (l == 0 && dx) ? dx : g[cur ^ 1];
    float* Gs = s.scale ? R.Gk(0, NL - 1) : nullptr;
    float* Gt = s.shift ? R.Gk(s.scale, NL - 1) : nullptr;
    hipLaunchKernelGGL(pick_nj(D, k_wbwd_update<1>, k_wbwd_update<2>, k_wbwd_update<3>,
                               k_wbwd_update<4>),
                       dim3(R.wave_blocks), dim3(256), 0, st, g[cur], gin, R.Xs(l),
                       R.Os(l), gld, Gs, Gt,
                       gz_all && l > 0 ? gz_all + (int64_t)(l - 1) * B * D : nullptr, fq + l * D,
                       B, R.geom);
    if (s.nets) {
      R.nets_backward(l, l, gin);
      const int r = R.weight_grads(l, l, grads + (int64_t)l * R.PL);
      if (r != CNF_OK) return r;
    }
    cur ^= 1;
  }
  return check_launch();
}

// Reverse mode of the INVERSE transform (flows/flows.py:114-126, Flow.backward
// under autograd): step i runs layer l = L-1-i on z' = z_in[:, iq_l] (flip and
// rev_perm undone as a gather), x_T = (z'_T - t) e^{-s}, x_C = z'_C,
// ld -= sum s.  Slot i holds step i's gathered input.  Backward, per step:
//   g_{z'_T} = g_T e^{-s},  G_t = -g_T e^{-s},  G_s = -g_T x_T - gld,
//   g_{z'_C} = g_C + (conditioners' share), then g_{z_in}[iq_l[j]] = g_{z'}[j]
//   plus the caller's gradient of the previous step's output.
// strict_nan: every feature follows the reference's op sequence (the strict
// branches of k_winv_stash / k_winv_fwd_update / k_winv_bwd_update), the nets
// see all D columns of x_b and write s, t for all D (lin_in / lin_out).
int wvjp_inv_run(const Shape& s, const void* prepared, const float* z, const float* gx,
                 const float* gx_all, const float* gld_in, float* grads, float* dz, int64_t B,
                 void* ws, size_t ws_bytes, hipStream_t st) {
  if (!wvjp_ok(s)) return CNF_ERR_UNSUPPORTED;
  // (the workspace is wvjp_inv_workspace's: the layer-at-a-time plan)
  const Plan p = make_plan(s, B);
  if (!ws || ws_bytes < (size_t)p.total * 4) return CNF_ERR_NULL;
  if (B == 0) return empty_batch(s, grads, nullptr, st);
  Runner R(s, p, ws, prepared, B, st);
  const int32_t* iq = reinterpret_cast<const int32_t*>(prepared) + s.L * s.D;
  const int D = s.D, NL = s.n_lin, L = s.L;
  float* W = R.W;
  float* gld = W + p.gld;

  // ---- forward sweep (the inverse): slot i = gathered input of step i ----
  hipLaunchKernelGGL(k_winv_stash, dim3(R.wave_blocks), dim3(256), 0, st, z, iq + (L - 1) * D,
                     R.Xs(0), B, R.geom);
  for (int i = 0; i < L; ++i) {
    const int l = L - 1 - i;
    if (s.nets) R.nets_forward(i, l);
    if (i + 1 < L)
      hipLaunchKernelGGL(k_winv_fwd_update, dim3(R.wave_blocks), dim3(256), 0, st, R.Xs(i),
                         R.Xs(i + 1), R.Os(i), R.Ot(i), iq + (l - 1) * D, B, R.geom);
  }
  // ---- seed: gradient of the last step's output (the flow's input estimate) ----
  float* g[2] = {W + p.g0, W + p.g1};
  float* tmp = W + p.g0;  // reuse: g ping-pongs between g1 and tmp below
  hipLaunchKernelGGL(k_wseed, dim3((unsigned)p.nseed), dim3(256), 0, st, R.Xs(0), gld, nullptr,
                     -1, 0.f, 1.f, gx, gx_all ? gx_all + (int64_t)(L - 1) * B * D : nullptr,
                     gld_in, g[1], gld, W + p.seed, B, R.geom);
  if (R.PL > 0 && hipMemsetAsync(W + p.part, 0, (size_t)p.nkb * R.PS * 4, st) != hipSuccess)
    return check_launch();

  // ---- backward sweep over the steps, last first ----
  for (int i = L - 1; i >= 0; --i) {
    const int l = L - 1 - i;
    if (s.nets && !p.keep_acts) R.nets_forward(i, l);
    float* Gs = s.scale ? R.Gk(0, NL - 1) : nullptr;
    float* Gt = s.shift ? R.Gk(s.scale, NL - 1) : nullptr;
    hipLaunchKernelGGL(k_winv_bwd_update, dim3(R.wave_blocks), dim3(256), 0, st, g[1], tmp,
                       R.Xs(i), R.Os(i), R.Ot(i), gld, Gs, Gt, B, R.geom);
    if (s.nets) {
      R.nets_backward(i, l, tmp);
      const int r = R.weight_grads(i, l, grads + (int64_t)l * R.PL);
      if (r != CNF_OK) return r;
    }
    hipLaunchKernelGGL(k_winv_scatter, dim3(R.wave_blocks), dim3(256), 0, st, tmp,
                       i == 0 ? dz : g[1],
                       gx_all && i > 0 ? gx_all + (int64_t)(i - 1) * B * D : nullptr,
                       iq + l * D, B, D, i == 0 && dz == nullptr);
  }
  return check_launch();
}

}  // namespace cnf
