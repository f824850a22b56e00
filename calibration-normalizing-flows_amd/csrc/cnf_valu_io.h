// Tile I/O and loss helpers shared by the narrow-flow forward kernels
// (cnf_valu.hip: LDS / scalar weights; cnf_sgpr.hip: pipelined scalar weights).
// A block owns a tile of ROWS*RW rows staged through LDS, so global loads and
// stores are 16-byte-per-lane coalesced sweeps; a lane holds RW rows.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "cnf_valu_common.h"

#ifndef CNF_VALU_NT_STORE
#define CNF_VALU_NT_STORE 1  // A/B: 0 = default-policy 16-B tile stores
#endif
#ifndef CNF_VALU_NT_LOAD
#define CNF_VALU_NT_LOAD 0  // A/B: streaming 16-B tile loads (every-layer pass 59.6 -> 65.1 us)
#endif

namespace cnf {
namespace valu {

// Block barrier for LDS hand-offs only: waits for this wave's LDS traffic,
// not for its outstanding global loads/stores (a __syncthreads() would also
// drain vmcnt, serialising the prefetch and the output stores).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int ROWS>
__device__ __forceinline__ void tile_load(float* __restrict__ sm, const float* __restrict__ src,
                                          int n, bool vec) {
  const int tid = threadIdx.x;
  int done = 0;
  if (vec) {
    const int n4 = n >> 2;
    float4* d4 = reinterpret_cast<float4*>(sm);
#if CNF_VALU_NT_LOAD
    typedef float nt4 __attribute__((ext_vector_type(4)));
    const nt4* s4 = reinterpret_cast<const nt4*>(src);
    for (int i = tid; i < n4; i += ROWS) {
      const nt4 q = __builtin_nontemporal_load(s4 + i);
      d4[i] = float4{q.x, q.y, q.z, q.w};
    }
#else
    const float4* s4 = reinterpret_cast<const float4*>(src);
    for (int i = tid; i < n4; i += ROWS) d4[i] = s4[i];
#endif
    done = n4 << 2;
  }
  for (int i = done + tid; i < n; i += ROWS) sm[i] = src[i];
}

template <int ROWS>
__device__ __forceinline__ void tile_store(float* __restrict__ dst, const float* __restrict__ sm,
                                           int n, bool vec) {
  const int tid = threadIdx.x;
  int done = 0;
  if (vec) {
    const int n4 = n >> 2;
    const float4* s4 = reinterpret_cast<const float4*>(sm);
#if CNF_VALU_NT_STORE
    // streaming stores: the rows are written once and never re-read here
    // (every-layer pass at 2^20 rows 70.4 -> 57.4 us)
    typedef float nt4 __attribute__((ext_vector_type(4)));
    nt4* d4 = reinterpret_cast<nt4*>(dst);
    for (int i = tid; i < n4; i += ROWS) {
      const float4 q = s4[i];
      __builtin_nontemporal_store(nt4{q.x, q.y, q.z, q.w}, d4 + i);
    }
#else
    float4* d4 = reinterpret_cast<float4*>(dst);
    for (int i = tid; i < n4; i += ROWS) d4[i] = s4[i];
#endif
    done = n4 << 2;
  }
  for (int i = done + tid; i < n; i += ROWS) dst[i] = sm[i];
}

// lane value <-> the RW rows a thread owns (rows tid and tid + ROWS of the tile)
template <int ROWS>
__device__ __forceinline__ float get_row(const float* sm, int i, int D, int k, float) {
  return sm[i * D + k];
}
template <int ROWS, class V>
__device__ __forceinline__ V get_row(const float* sm, int i, int D, int k, V) {
  V r;
#pragma unroll
  for (int q = 0; q < (int)(sizeof(V) / sizeof(float)); ++q) r[q] = sm[(i + q * ROWS) * D + k];
  return r;
}
template <int ROWS>
__device__ __forceinline__ void put_row(float* sm, int i, int D, int k, float v) {
  sm[i * D + k] = v;
}
template <int ROWS, class V>
__device__ __forceinline__ void put_row(float* sm, int i, int D, int k, V v) {
#pragma unroll
  for (int q = 0; q < (int)(sizeof(V) / sizeof(float)); ++q) sm[(i + q * ROWS) * D + k] = v[q];
}

// Write the tile's rows (registers in orientation O) to dst through LDS.
template <int D, int ROWS, bool O, class T>
__device__ __forceinline__ void store_rows(float* __restrict__ dst, float* sm, const T* v,
                                           int nrows, bool vec) {
  const int tid = threadIdx.x;
  lds_barrier();  // previous users of sm are done
#pragma unroll
  for (int j = 0; j < D; ++j) put_row<ROWS>(sm, tid, D, j, v[R<D, O>(j)]);
  lds_barrier();
  tile_store<ROWS>(dst, sm, nrows * D, vec);
}

__device__ __forceinline__ float comp(float v, int) { return v; }
template <class V>
__device__ __forceinline__ float comp(V v, int q) { return v[q]; }

// Write the lane's RW rows (registers in orientation O) straight to dst: one
// 8-B store per pair of logits when D is even and dst is 8-B aligned, else
// one 4-B store per logit.  A wave-instruction covers 64 consecutive rows, so
// L2 sees whole lines across the row's few stores; no LDS, no barrier.
template <int D, int ROWS, bool O, class T>
__device__ __forceinline__ void store_rows_direct(float* __restrict__ dst, const T* v, int nrows,
                                                  bool al8) {
  constexpr int RW = sizeof(T) / sizeof(float);
  const int tid = threadIdx.x;
#pragma unroll
  for (int q = 0; q < RW; ++q) {
    const int r = tid + q * ROWS;
    if (r >= nrows) continue;
    float* d = dst + (int64_t)r * D;
    if (D % 2 == 0 && al8) {
#pragma unroll
      for (int j = 0; j < D; j += 2)
        *reinterpret_cast<float2*>(d + j) =
            float2{comp(v[R<D, O>(j)], q), comp(v[R<D, O>(j + 1)], q)};
    } else {
#pragma unroll
      for (int j = 0; j < D; ++j) d[j] = comp(v[R<D, O>(j)], q);
    }
  }
}

// Loss terms of the tile's rows (registers in orientation O, RW rows per lane):
// CAL: loss = -(log(softmax(z)[y] + 1e-7) + ld)       calibrators.py:288-291
// CE:  loss = -log_softmax(z)[y] - det * ld            run_experiment3D.py:107
// The max / shifted-exp / sum run on whole RW-row vectors (packed FMAs);
// z[y] is picked per row by sel_tree (below).
// Labels of the lane's RW rows (low 32-bit word of the int64 targets; -1 past
// the batch end), issued with the tile load so the latency hides under the
// layer sweep instead of stalling the loss at the end.
template <int RW>
__device__ __forceinline__ void load_labels(const int64_t* __restrict__ yl, int64_t row0, int tid,
                                            int rows, int64_t B, int* y) {
  const int32_t* y32 = reinterpret_cast<const int32_t*>(yl);
#pragma unroll
  for (int q = 0; q < RW; ++q) {
    const int64_t row = row0 + tid + (int64_t)q * rows;
    y[q] = row < B ? y32[2 * row] : -1;
  }
}

// z[y] by a binary select tree on the label's bits, all integer bit work:
// per level one v_bfe_i32 turns bit b of y into a 0 / -1 mask and each pair is
// merged by one v_bfi_b32 -- ceil(log2 D) + D - 1 VALU per row, no lane masks
// (so no VCC hazard nops), no branches, and no select chain for LLVM to fold
// into a scratch-indexed load.  Labels outside [0, D) pick 0, as a linear
// scan would.
template <int N>
__device__ __forceinline__ uint32_t sel_tree(const uint32_t* a, int y, int bit) {
  if constexpr (N == 1) {
    return a[0];
  } else {
    constexpr int M = (N + 1) / 2;
    uint32_t b[M];
    const uint32_t m = (uint32_t)((y << (31 - bit)) >> 31);  // arithmetic: 0 or ~0
#pragma unroll
    for (int p = 0; p < N / 2; ++p) b[p] = (m & a[2 * p + 1]) | (~m & a[2 * p]);
    if constexpr (N & 1) b[M - 1] = a[N - 1];
    return sel_tree<M>(b, y, bit + 1);
  }
}

template <int D, bool O, class T>
__device__ __forceinline__ void tile_loss(const T* v, T ld, const int* y, int kind, float det,
                                          float& t0, float& t1, float& t2) {
  constexpr int RW = sizeof(T) / sizeof(float);
  constexpr float kL2E = 1.4426950408889634f, kLN2 = 0.6931471805599453f;
  T m = v[R<D, O>(0)];
#pragma unroll
  for (int j = 1; j < D; ++j) m = maxT(m, v[R<D, O>(j)]);
  const T nm = m * splat(-kL2E, T{});
  T se = splat(0.f, T{}), zy = splat(0.f, T{});
#pragma unroll
  for (int j = 0; j < D; ++j) se += exp2T(fmaT(kL2E, v[R<D, O>(j)], nm));
#pragma unroll
  for (int q = 0; q < RW; ++q) {
    uint32_t zq[D];
#pragma unroll
    for (int j = 0; j < D; ++j) zq[j] = __float_as_uint(comp(v[R<D, O>(j)], q));
    const float pk = __uint_as_float(sel_tree<D>(zq, y[q], 0));
    setc(zy, q, (unsigned)y[q] < (unsigned)D ? pk : 0.f);
  }
#pragma unroll
  for (int q = 0; q < RW; ++q) {
    if (y[q] < 0) continue;
    const float lpy = comp(zy, q) - (comp(m, q) + __builtin_amdgcn_logf(comp(se, q)) * kLN2);
    const float l = comp(ld, q);
    float ce, loss;
    if (kind == CNF_LOSS_CAL) {
      ce = -__builtin_amdgcn_logf(__builtin_amdgcn_exp2f(lpy * kL2E) + 1e-7f) * kLN2;
      loss = ce - l;
    } else {
      ce = -lpy;
      loss = ce - det * l;
    }
    t0 += loss;
    t1 += ce;
    t2 += l;
  }
}

// Block sum of three per-thread values in a fixed order -> part[blockIdx][0..2]
// (plain stores; the wave exits right after).  The host side adds the
// partials in block order with one small follow-up launch (reduce_partials),
// so the fused eval stays deterministic without any block waiting on a
// device-scope hand-off.
// Wave sum into lane 63 by DPP (row_shr 1/2/4/8 inside each 16-lane row,
// then row_bcast 15 / 31 across rows): VALU ops with a few cycles of latency
// each, where the xor butterfly's __shfl_xor is six dependent ds_bpermute
// round trips through LDS.  Only lane 63's result is meaningful.
__device__ __forceinline__ float wave_sum_dpp63(float v) {
  auto dpp = [](float x, auto ctl) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
        0, __builtin_bit_cast(int, x), decltype(ctl)::value, 0xf, 0xf, false));
  };
  v += dpp(v, std::integral_constant<int, 0x111>{});  // row_shr:1
  v += dpp(v, std::integral_constant<int, 0x112>{});  // row_shr:2
  v += dpp(v, std::integral_constant<int, 0x114>{});  // row_shr:4
  v += dpp(v, std::integral_constant<int, 0x118>{});  // row_shr:8
  v += dpp(v, std::integral_constant<int, 0x142>{});  // row_bcast:15
  v += dpp(v, std::integral_constant<int, 0x143>{});  // row_bcast:31
  return v;
}

template <int ROWS>
__device__ __forceinline__ void block_sum3(float a, float b, float c, float* sm, float* part) {
  a = wave_sum_dpp63(a);
  b = wave_sum_dpp63(b);
  c = wave_sum_dpp63(c);
  const int tid = threadIdx.x, w = tid >> 6;
  constexpr int kLead = 63;  // the lane holding the wave's sums
  lds_barrier();
  if ((tid & 63) == kLead) {
    sm[4 * w] = a;
    sm[4 * w + 1] = b;
    sm[4 * w + 2] = c;
  }
  lds_barrier();
  if (tid == 0) {
    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
    for (int i = 0; i < ROWS / 64; ++i) {
      s0 += sm[4 * i];
      s1 += sm[4 * i + 1];
      s2 += sm[4 * i + 2];
    }
    reinterpret_cast<float4*>(part)[blockIdx.x] = float4{s0, s1, s2, 0.f};
  }
}


// The loss-term sums of nblk 16-B partial records by one 256-thread block
// (threadIdx.x = t), in ONE fixed order: lane-strided sums with up to eight
// records per lane in flight, a DPP sum per wave, waves in index order
// (k_reduce_rows4, the follow-up launch of the fused eval passes).
// An in-launch sum measured slower both ways it was tried (round 5-6,
// DESIGN.md section 3): the last block found by a counter that every block
// adds to (~1,500 returning atomics on one word at the end of a 2^20-row
// call, +4.4 us), and a reducer block polling every block's tagged record
// (no atomics, +0.3 us: the hand-off's latency equals the launch boundary).
constexpr int kRR = 256;
__device__ __forceinline__ void reduce_rows4_block(const float4* __restrict__ partials, int nblk,
                                                   float* __restrict__ out, float (*red)[3]) {
  const int t = threadIdx.x;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f;
  for (int b0 = t; b0 < nblk; b0 += 8 * kRR) {
    float4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int b = b0 + k * kRR;
      v[k] = b < nblk ? partials[b] : float4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      s0 += v[k].x;
      s1 += v[k].y;
      s2 += v[k].z;
    }
  }
  s0 = wave_sum_dpp63(s0);
  s1 = wave_sum_dpp63(s1);
  s2 = wave_sum_dpp63(s2);
  constexpr int kLead = 63;
  if ((t & 63) == kLead) {
    red[t >> 6][0] = s0;
    red[t >> 6][1] = s1;
    red[t >> 6][2] = s2;
  }
  __syncthreads();
  if (t < 3) {
    float a = 0.f;
#pragma unroll
    for (int w = 0; w < kRR / 64; ++w) a += red[w][t];
    out[t] = a;
  }
}

template <int ROWS>
__device__ __forceinline__ void store_ld(float* ld_out, int64_t row0, int tid, int nrows, float v) {
  if (tid < nrows) ld_out[row0 + tid] = v;
}
template <int ROWS, class V>
__device__ __forceinline__ void store_ld(float* ld_out, int64_t row0, int tid, int nrows, V v) {
#pragma unroll
  for (int q = 0; q < (int)(sizeof(V) / sizeof(float)); ++q)
    if (tid + q * ROWS < nrows) ld_out[row0 + tid + q * ROWS] = v[q];
}

}  // namespace valu
}  // namespace cnf
