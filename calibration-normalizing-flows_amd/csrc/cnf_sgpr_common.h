// Pipelined-SGPR weight path and wave-tile I/O shared by the narrow-flow
// kernels that carry a lane's rows as packed pairs: k_sgpr (cnf_sgpr.hip,
// forward / inverse / loss / predict) and k_vjp2 (cnf_vjp.hip, reverse mode).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "cnf_valu_common.h"

namespace cnf {
namespace valu {

// Compile-time layout of one net in the packed-SGPR region (must match
// derive_shape's sp_lin_off and cnf_prepare's mode 3).
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
// multiplier and the high half as the addend, so the bias costs no VALU move.
__device__ __forceinline__ f2 fma_wb(f2 wb, f2 x) {
  f2 a;
  asm("v_pk_fma_f32 %0, %1, %2, %1 op_sel:[0,0,1] op_sel_hi:[0,1,1]" : "=v"(a) : "s"(wb), "v"(x));
  return a;
}
// ... and the clamped forms that end a hidden neuron (relu folded, see header)
__device__ __forceinline__ f2 fma_wb_clamp(f2 wb, f2 x) {
  f2 a;
  asm("v_pk_fma_f32 %0, %1, %2, %1 op_sel:[0,0,1] op_sel_hi:[0,1,1] clamp"
      : "=v"(a) : "s"(wb), "v"(x));
  return a;
}
__device__ __forceinline__ f2 fma_clamp(float w, f2 x, f2 acc) {
  f2 a;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1] clamp" : "=v"(a) : "s"(f2{w, w}), "v"(x),
      "v"(acc));
  return a;
}

// acc + w * x with w = weights[idx] broadcast to both packed lanes straight
// from the aligned SGPR pair holding it: op_sel / op_sel_hi pick that pair's
// element for both lanes.  (A plain fma of a float weight made the compiler
// copy each odd-indexed weight into a scratch even pair first; when the
// scratch pair was part of the next block's in-flight s_load destination, it
// had to wait for that load -- a full scalar-load latency inside a Linear.)
template <int NC>
__device__ __forceinline__ f2 fma_ws(const SW<NC>& w, int idx, f2 x, f2 acc) {
  const f2 p = w.pair(idx & ~1);
  f2 a;
  if (idx & 1)
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,1,1]"
        : "=v"(a) : "s"(p), "v"(x), "v"(acc));
  else
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]" : "=v"(a) : "s"(p), "v"(x), "v"(acc));
  return a;
}
template <int NC>
__device__ __forceinline__ f2 fma_ws_clamp(const SW<NC>& w, int idx, f2 x, f2 acc) {
  const f2 p = w.pair(idx & ~1);
  f2 a;
  if (idx & 1)
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,1,1] clamp"
        : "=v"(a) : "s"(p), "v"(x), "v"(acc));
  else
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1] clamp"
        : "=v"(a) : "s"(p), "v"(x), "v"(acc));
  return a;
}

// w * x, w = weights[idx] broadcast from its aligned SGPR pair (as fma_ws)
template <int NC>
__device__ __forceinline__ f2 mul_ws(const SW<NC>& w, int idx, f2 x) {
  const f2 p = w.pair(idx & ~1);
  f2 a;
  if (idx & 1)
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1]" : "=v"(a) : "s"(p), "v"(x));
  else
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(a) : "s"(p), "v"(x));
  return a;
}

// Weight-block loads.  Each Linear's block arrives in SGPRs one Linear ahead:
//   sready()          wait for the block issued one Linear ago -- a
//                     compiler-visible s_waitcnt lgkmcnt(0), so the compiler
//                     adds no wait of its own before the block's first use
//                     (scalar loads return out of order: any later wait
//                     would be lgkmcnt(0) and would also wait for the block
//                     issued next);
//   sissue(next, p)   then issue the next block, before this Linear's FMAs.
// Plain (compiler-visible) loads: the waitcnt pass guards every read of the
// destination SGPRs, copies and spills included.  The sched_barriers pin the
// order wait -> issue -> FMAs, and leave each Linear's neurons one scheduling
// region.  (An inline-asm load/wait pair let the register allocator copy
// still-in-flight SGPRs.)
__device__ __forceinline__ void sready() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0); vmcnt, expcnt untouched (gfx9 encoding)
  __builtin_amdgcn_sched_barrier(0);
}
template <int NC>
__device__ __forceinline__ void sissue(SW<NC>& r, const float* p) {
  const v16f* q = reinterpret_cast<const v16f*>(__builtin_assume_aligned(p, 64));
#pragma unroll
  for (int i = 0; i < NC; ++i) r.c[i] = q[i];
  __builtin_amdgcn_sched_barrier(0);
}

// HBM -> LDS copy of one full wave tile (TR*D floats, 16-B aligned) by
// LDS-DMA: one global_load_lds_dwordx4 moves 1 KiB, lane-linear.
// kDmaAux: the loads' cache-policy bits (gfx950: 1 sc0, 2 nt, 16 sc1).
// Streaming (nt) input: the cfg2 pass is held at the board's power cap
// (1.4 kW at 2^23 rows; tools/power_probe.py), and the nt DMA takes 8 % less
// energy per row than the default policy -- 31.39 -> 30.24 us per 2^20-row
// loss call, 192.8 -> 188.9 us at 2^23, outputs bitwise unchanged (round 5,
// profiles/r05_ab_power.jsonl); sc1 nt measured the same as nt.
constexpr int kDmaAux = 2;
template <int D, int TR>
__device__ __forceinline__ void wave_dma(float* sm, const float* __restrict__ src, int lane) {
  constexpr int N4 = TR * D / 4, NI = (N4 + 63) / 64;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    if (N4 % 64 == 0 || i * 64 + lane < N4)
      __builtin_amdgcn_global_load_lds(src + (i * 64 + lane) * 4,
                                       (__attribute__((address_space(3))) void*)(sm + i * 256), 16,
                                       0, kDmaAux);
  }
}

// the lane's pairs from the LDS tile (one ds_read2_b32 per feature and pair)
// (REV: feature k lands in v[p][D-1-k], the row held reversed)
template <int D, int P, bool REV = false>
__device__ __forceinline__ void read_pairs(const float* sm, int lane, f2 (&v)[P][D]) {
  const float* b = sm + 2 * P * D * lane;
#pragma unroll
  for (int p = 0; p < P; ++p)
#pragma unroll
    for (int k = 0; k < D; ++k)
      v[p][REV ? D - 1 - k : k] = f2{b[2 * p * D + k], b[(2 * p + 1) * D + k]};
}

// ds_read2_pairs<D>(base, o): o[k] = (lds[base + k], lds[base + D + k]) for
// k < D -- D ds_read2_b32 straight into the pair registers AND the wait for
// them in ONE asm statement, so the compiler never sees a pair register
// before its data has landed (a wait in a separate statement would leave it
// free to copy or spill a register between the read and the wait).  Outputs
// are early-clobber: no pair may share the address register.  One
// specialisation per D (an asm string's length is fixed).
#define CNF_RP_L(k) "ds_read2_b32 %" #k ", %[b] offset0:" #k " offset1:%[d]+" #k "\n\t"
#define CNF_RP_O(k) "=&v"(o[k])
#define CNF_RPL2 CNF_RP_L(0) CNF_RP_L(1)
#define CNF_RPL3 CNF_RPL2 CNF_RP_L(2)
#define CNF_RPL4 CNF_RPL3 CNF_RP_L(3)
#define CNF_RPL5 CNF_RPL4 CNF_RP_L(4)
#define CNF_RPL6 CNF_RPL5 CNF_RP_L(5)
#define CNF_RPL7 CNF_RPL6 CNF_RP_L(6)
#define CNF_RPL8 CNF_RPL7 CNF_RP_L(7)
#define CNF_RPL9 CNF_RPL8 CNF_RP_L(8)
#define CNF_RPL10 CNF_RPL9 CNF_RP_L(9)
#define CNF_RPL11 CNF_RPL10 CNF_RP_L(10)
#define CNF_RPL12 CNF_RPL11 CNF_RP_L(11)
#define CNF_RPL13 CNF_RPL12 CNF_RP_L(12)
#define CNF_RPL14 CNF_RPL13 CNF_RP_L(13)
#define CNF_RPL15 CNF_RPL14 CNF_RP_L(14)
#define CNF_RPL16 CNF_RPL15 CNF_RP_L(15)
#define CNF_RPO2 CNF_RP_O(0), CNF_RP_O(1)
#define CNF_RPO3 CNF_RPO2, CNF_RP_O(2)
#define CNF_RPO4 CNF_RPO3, CNF_RP_O(3)
#define CNF_RPO5 CNF_RPO4, CNF_RP_O(4)
#define CNF_RPO6 CNF_RPO5, CNF_RP_O(5)
#define CNF_RPO7 CNF_RPO6, CNF_RP_O(6)
#define CNF_RPO8 CNF_RPO7, CNF_RP_O(7)
#define CNF_RPO9 CNF_RPO8, CNF_RP_O(8)
#define CNF_RPO10 CNF_RPO9, CNF_RP_O(9)
#define CNF_RPO11 CNF_RPO10, CNF_RP_O(10)
#define CNF_RPO12 CNF_RPO11, CNF_RP_O(11)
#define CNF_RPO13 CNF_RPO12, CNF_RP_O(12)
#define CNF_RPO14 CNF_RPO13, CNF_RP_O(13)
#define CNF_RPO15 CNF_RPO14, CNF_RP_O(14)
#define CNF_RPO16 CNF_RPO15, CNF_RP_O(15)
template <int D>
__device__ __forceinline__ void ds_read2_pairs(uint32_t base, f2* o);
#define CNF_RPW(D)                                                                   \
  template <>                                                                        \
  __device__ __forceinline__ void ds_read2_pairs<D>(uint32_t base, f2 * o) {         \
    asm volatile(CNF_RPL##D "s_waitcnt lgkmcnt(0)"                                   \
                 : CNF_RPO##D                                                        \
                 : [b] "v"(base), [d] "i"(D)                                         \
                 : "memory");                                                        \
  }
CNF_RPW(2) CNF_RPW(3) CNF_RPW(4) CNF_RPW(5) CNF_RPW(6) CNF_RPW(7) CNF_RPW(8) CNF_RPW(9)
CNF_RPW(10) CNF_RPW(11) CNF_RPW(12) CNF_RPW(13) CNF_RPW(14) CNF_RPW(15) CNF_RPW(16)
#undef CNF_RPW

// read_pairs with the ds_read2_b32 issued straight into the pair registers
// and waited for in the same asm statement (ds_read2_pairs).  (The compiler
// merged the plain loads into ds_read_b128 of four features of one row, and
// regrouping those into pairs cost ~15 v_mov per tile.)
template <int D, bool REV = false>
__device__ __forceinline__ void read_pairs_wait(const float* sm, int lane, f2 (&v)[1][D]) {
  static_assert(D >= 2 && D <= 16, "ds_read2_pairs is specialised for 2 <= D <= 16");
  typedef __attribute__((address_space(3))) const float lds_f;
  const uint32_t base = (uint32_t)(uintptr_t)(lds_f*)(sm + 2 * D * lane);
  f2 o[D];
  ds_read2_pairs<D>(base, o);
#pragma unroll
  for (int k = 0; k < D; ++k) v[0][REV ? D - 1 - k : k] = o[k];
}

// Coalesced tile stores.  A lane's 2P output rows sit 2*P*D floats apart from
// the next lane's, so storing them straight from registers makes every 16-B
// store instruction touch 64 scattered pieces of ~40 cache lines (partial-line
// writes the L2 must merge; measured: writing z cost 5.5 us of a 39 us cfg2
// pass).  Instead the lane writes its rows into the wave's LDS tile (row-major,
// the input tile's layout) and the wave stores the tile lane-linear: each
// global_store_dwordx4 then writes 1 KiB contiguous (8 whole lines).
// One ds_write2_b32 per feature and pair writes the pair's two halves
// straight into their rows (the mirror of read_pairs' ds_read2_b32); plain
// stores were merged into ds_write_b128 of four features of one row, which
// costs a v_mov per float to regroup the pair registers.  LDS operations of a
// wave complete in issue order, so the tile reads that follow need no wait;
// the "memory" clobber keeps the compiler from moving them above the writes.
template <int D, int P>
__device__ __forceinline__ void stage_pairs(float* sm, int lane, const f2 (&v)[P][D]) {
  static_assert(2 * P * D <= 256, "ds_write2_b32 dword offsets are 8-bit");
  typedef __attribute__((address_space(3))) float lds_f;
  const uint32_t base = (uint32_t)(uintptr_t)(lds_f*)(sm + 2 * P * D * lane);
#pragma unroll
  for (int p = 0; p < P; ++p)
#pragma unroll
    for (int k = 0; k < D; ++k)
      asm volatile("ds_write2_b32 %0, %1, %2 offset0:%3 offset1:%4"
                   :
                   : "v"(base), "v"(v[p][k].x), "v"(v[p][k].y), "i"(2 * p * D + k),
                     "i"((2 * p + 1) * D + k)
                   : "memory");
}
template <int TF>
__device__ __forceinline__ void store_tile(float* __restrict__ dst, const float* sm, int lane) {
  constexpr int N4 = TF / 4, NI = (N4 + 63) / 64;
  static_assert(TF % 4 == 0, "tile must be whole float4s");
  float4 q[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i)
    if (N4 % 64 == 0 || i * 64 + lane < N4)
      q[i] = *reinterpret_cast<const float4*>(sm + (i * 64 + lane) * 4);
#pragma unroll
  for (int i = 0; i < NI; ++i)
    if (N4 % 64 == 0 || i * 64 + lane < N4) {
      // streaming (nt) stores.  Write-through (sc1, sc0 sc1, sc1 nt) measured
      // 28-49 % slower per 2^20-row call (round 6): the stores then wait on
      // the fabric instead of draining from L2
      using v4 = __attribute__((ext_vector_type(4))) float;
      __builtin_nontemporal_store(v4{q[i].x, q[i].y, q[i].z, q[i].w},
                                  reinterpret_cast<v4*>(dst) + i * 64 + lane);
    }
}

// The lane's 2*P*D output floats (pairs in logical order) to dst = its first
// row: 16-B stores when aligned, else 8-B, else 4-B; `rows` < 2P on the ragged
// tile.
template <int D, int P>
__device__ __forceinline__ void store_rows(float* __restrict__ dst, const f2 (&v)[P][D], int rows,
                                           int al) {
  constexpr int NF = 2 * P * D;
  float r[NF];
#pragma unroll
  for (int p = 0; p < P; ++p)
#pragma unroll
    for (int k = 0; k < D; ++k) {
      r[2 * p * D + k] = v[p][k].x;
      r[(2 * p + 1) * D + k] = v[p][k].y;
    }
  if (rows == 2 * P && NF % 4 == 0 && al >= 16) {
#pragma unroll
    for (int q = 0; q < NF / 4; ++q)
      reinterpret_cast<float4*>(dst)[q] = float4{r[4 * q], r[4 * q + 1], r[4 * q + 2], r[4 * q + 3]};
  } else if (rows == 2 * P && NF % 2 == 0 && al >= 8) {
#pragma unroll
    for (int q = 0; q < NF / 2; ++q) reinterpret_cast<float2*>(dst)[q] = float2{r[2 * q], r[2 * q + 1]};
  } else {
#pragma unroll
    for (int k = 0; k < NF; ++k)
      if (k < rows * D) dst[k] = r[k];
  }
}

template <int P>
__device__ __forceinline__ void store_lds(float* __restrict__ dst, const f2 (&ld)[P], int rows,
                                          int al) {
  if (P == 2 && rows == 4 && al >= 16) {
    *reinterpret_cast<float4*>(dst) = float4{ld[0].x, ld[0].y, ld[P - 1].x, ld[P - 1].y};
  } else if (rows == 2 * P && al >= 8) {
#pragma unroll
    for (int p = 0; p < P; ++p) {
      reinterpret_cast<float2*>(dst)[p] = float2{ld[p].x, ld[p].y};
    }
  } else {
#pragma unroll
    for (int p = 0; p < P; ++p) {
      if (2 * p < rows) dst[2 * p] = ld[p].x;
      if (2 * p + 1 < rows) dst[2 * p + 1] = ld[p].y;
    }
  }
}

// reverse the logical order of a row held in orientation 1 (odd L): afterwards
// v[j] is logical j, so the epilogues have one form
template <int D>
__device__ __forceinline__ void unflip(f2* v) {
#pragma unroll
  for (int k = 0; k < D / 2; ++k) {
    const f2 a = v[k];
    v[k] = v[D - 1 - k];
    v[D - 1 - k] = a;
  }
}

// Labels of the lane's rows (int64 each, 16-B loads when aligned), packed one
// byte per row into ONE register so they cost no VGPRs across the layer sweep.
// A label is valid iff 0 <= y < D; an invalid one (byte 0xff) poisons the loss
// terms with NaN (the reference's probs.gather raises on it).  rows: valid rows.
template <int D, int P>
__device__ __forceinline__ uint32_t load_labels(const int64_t* __restrict__ y, int rows,
                                                bool al16) {
  uint32_t packed = 0;
  const int32_t* y32 = reinterpret_cast<const int32_t*>(y);
#pragma unroll
  for (int p = 0; p < P; ++p) {
    int lo0 = 0, hi0 = 0, lo1 = 0, hi1 = 0;
    if (rows == 2 * P && al16) {
      const int4 q = reinterpret_cast<const int4*>(y32)[p];
      lo0 = q.x, hi0 = q.y, lo1 = q.z, hi1 = q.w;
    } else {
      if (2 * p < rows) lo0 = y32[4 * p], hi0 = y32[4 * p + 1];
      if (2 * p + 1 < rows) lo1 = y32[4 * p + 2], hi1 = y32[4 * p + 3];
    }
    const uint32_t b0 = hi0 == 0 && (unsigned)lo0 < (unsigned)D ? (uint32_t)lo0 : 0xffu;
    const uint32_t b1 = hi1 == 0 && (unsigned)lo1 < (unsigned)D ? (uint32_t)lo1 : 0xffu;
    packed |= (b0 | (b1 << 8)) << (16 * p);
  }
  return packed;
}

}  // namespace valu
}  // namespace cnf
