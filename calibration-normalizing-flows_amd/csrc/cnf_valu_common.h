// Device helpers shared by the narrow-flow (VALU, one logit vector per lane)
// kernels: forward/inverse (cnf_valu.hip) and reverse mode (cnf_vjp.hip).
// Shapes are compile-time so every weight offset is a constant and weight
// reads are wave-uniform scalar loads.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "cnf_internal.h"

namespace cnf {
namespace valu {

// A lane carries RW logit vectors: T = float (RW = 1) or an ext_vector of RW
// floats.  Every weight is a wave-uniform scalar (SGPR) shared by the RW
// vectors, so RW divides the scalar-cache traffic per vector.
typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <int RW> struct RowT { typedef float type; };
template <> struct RowT<2> { typedef f2 type; };
template <> struct RowT<4> { typedef f4 type; };

__device__ __forceinline__ float splat(float w, float) { return w; }
template <class V>
__device__ __forceinline__ V splat(float w, V) { return V(w); }
__device__ __forceinline__ float maxT(float a, float b) { return fmaxf(a, b); }
template <class V>
__device__ __forceinline__ V maxT(V a, V b) { return __builtin_elementwise_max(a, b); }
__device__ __forceinline__ float exp2T(float x) { return __builtin_amdgcn_exp2f(x); }
template <class V>
__device__ __forceinline__ V exp2T(V x) {
  V r;
#pragma unroll
  for (int i = 0; i < (int)(sizeof(V) / sizeof(float)); ++i) r[i] = __builtin_amdgcn_exp2f(x[i]);
  return r;
}
__device__ __forceinline__ void setc(float& v, int, float x) { v = x; }
template <class V>
__device__ __forceinline__ void setc(V& v, int q, float x) { v[q] = x; }
__device__ __forceinline__ float fmaT(float w, float x, float a) { return fmaf(w, x, a); }
template <class V>
__device__ __forceinline__ V fmaT(float w, V x, V a) { return __builtin_elementwise_fma(V(w), x, a); }
__device__ __forceinline__ f2 fmaT(f2 w, f2 x, f2 a) { return __builtin_elementwise_fma(w, x, a); }
__device__ __forceinline__ f2 splat(f2 w, f2) { return w; }
__device__ __forceinline__ float fmaV(float x, float y, float a) { return fmaf(x, y, a); }
template <class V>
__device__ __forceinline__ V fmaV(V x, V y, V a) { return __builtin_elementwise_fma(x, y, a); }

// FX: exp2(x*log2e) on v_exp_f32 (2 instructions; relative error ~|x|*6e-8
// + 1 ulp) instead of the range-reduced libm expf (~11 instructions).
template <bool FX>
__device__ __forceinline__ float expT(float x) { return FX ? __expf(x) : expf(x); }
template <bool FX, class V>
__device__ __forceinline__ V expT(V x) {
  V r;
#pragma unroll
  for (int i = 0; i < (int)(sizeof(V) / sizeof(float)); ++i) r[i] = expT<FX>(x[i]);
  return r;
}

template <bool STRICT>
__device__ __forceinline__ float relu(float a) {
  // torch.relu propagates NaN; v_max_f32 (IEEE maxNum) would drop it.
  if constexpr (STRICT) return a < 0.f ? 0.f : a;
  else return fmaxf(a, 0.f);
}
template <bool STRICT, class V>
__device__ __forceinline__ V relu(V a) {
  V r;
#pragma unroll
  for (int i = 0; i < (int)(sizeof(V) / sizeof(float)); ++i) r[i] = relu<STRICT>(a[i]);
  return r;
}

// Hidden activation of a conditioner Linear: ACT 0 none, 1 ReLU, 2 tanh (the
// legacy s-net, code-old/realNVP.py:61, CNF_OPT_S_TANH).
template <int ACT, bool STRICT>
__device__ __forceinline__ float act(float a) {
  if constexpr (ACT == 1) return relu<STRICT>(a);
  else if constexpr (ACT == 2) return tanhf(a);
  else return a;
}
template <int ACT, bool STRICT, class V>
__device__ __forceinline__ V act(V a) {
  V r;
#pragma unroll
  for (int i = 0; i < (int)(sizeof(V) / sizeof(float)); ++i) r[i] = act<ACT, STRICT>(a[i]);
  return r;
}

// Compact weight layout of the narrow-flow kernels (written by cnf_prepare):
// per Linear, W[NOUT][pad4(NIN)] row-major (zero padded), then b[pad4(NOUT)];
// the first Linear keeps only the NIN = D - D//2 conditioning columns (the
// masked input is zero elsewhere, flows/flows.py:102,105).  Every row and
// every block starts 16-B aligned, so 4 weights are one wide load.
__host__ __device__ constexpr int pad4(int x) { return (x + 3) & ~3; }

__host__ __device__ constexpr int pad16(int x) { return (x + 15) & ~15; }

template <int NIN, int NOUTF>
struct Lin {
  static constexpr int stride = pad4(NIN);
  // whole block padded to 64 B: weights are fetched as 16-float scalar chunks
  static constexpr int floats = pad16(NOUTF * pad4(NIN) + pad4(NOUTF));
};

// Weight i of a 64-B aligned block, read through 16-float (s_load_dwordx16)
// chunks so a Linear costs a few wide scalar-cache requests instead of one
// per 1-4 weights (the scalar cache's request rate bounds these kernels).
typedef float v16f __attribute__((ext_vector_type(16)));
__device__ __forceinline__ float wget(const float* __restrict__ w, int i) {
  return reinterpret_cast<const v16f*>(w)[i >> 4][i & 15];
}

// Weight i of a Linear block: float blobs read as wide scalar chunks; pair
// blobs (each weight stored twice, LDS) read as one 8-B element that is
// directly the packed operand of v_pk_fma_f32 for two vectors per lane.
__device__ __forceinline__ float wld(const float* __restrict__ w, int i) { return wget(w, i); }
__device__ __forceinline__ f2 wld(const f2* __restrict__ w, int i) { return w[i]; }

template <int D, int H1, int H2>
struct Net {
  static constexpr int DT = D / 2, DC = D - D / 2;
  static constexpr int floats = H1 == 0   ? Lin<DC, D>::floats
                                : H2 == 0 ? Lin<DC, H1>::floats + Lin<H1, D>::floats
                                          : Lin<DC, H1>::floats + Lin<H1, H2>::floats +
                                                Lin<H2, D>::floats;
};

// y[o] = act(b[o] (+p0) + sum_k W[o][k] * x[k]),  o < NOUT <= NOUTF.
template <int NIN, int NOUTF, int NOUT, int ACT, bool STRICT, bool POISON, class T, class WP>
__device__ __forceinline__ void linear(const WP* __restrict__ w, const T* x, T* y, T p0) {
  constexpr int S = Lin<NIN, NOUTF>::stride;
#pragma unroll
  for (int o = 0; o < NOUT; ++o) {
    T a = splat(wld(w, NOUTF * S + o), T{});
    if constexpr (POISON) a += p0;
#pragma unroll
    for (int k = 0; k < NIN; ++k) {
      a = fmaT(wld(w, o * S + k), x[k], a);
    }
    y[o] = act<ACT, STRICT>(a);
  }
}

// A whole Linear block (NCH 64-B chunks) fetched by ONE asm statement: NCH
// s_load_dwordx16 then a single wait, so the scalar cache sees NCH wide
// requests per Linear (hipcc otherwise narrows the loads to the elements it
// uses: many 4-16 B requests, and the scalar cache's request rate becomes
// the kernel's bound).
template <int NCH>
struct Chunks {
  v16f c[NCH];
  __device__ __forceinline__ float operator[](int i) const { return c[i >> 4][i & 15]; }
};

template <int NCH>
__device__ __forceinline__ Chunks<NCH> sload(const float* p) {
  Chunks<NCH> r;
  if constexpr (NCH == 1) {
    asm volatile("s_load_dwordx16 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)"
                 : "=s"(r.c[0]) : "s"(p));
  } else if constexpr (NCH == 2) {
    asm volatile("s_load_dwordx16 %0, %2, 0x0\n\ts_load_dwordx16 %1, %2, 0x40\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=s"(r.c[0]), "=s"(r.c[1]) : "s"(p));
  } else {
    static_assert(NCH == 3, "Linear block too large for the scalar-chunk path");
    asm volatile("s_load_dwordx16 %0, %3, 0x0\n\ts_load_dwordx16 %1, %3, 0x40\n\t"
                 "s_load_dwordx16 %2, %3, 0x80\n\ts_waitcnt lgkmcnt(0)"
                 : "=s"(r.c[0]), "=s"(r.c[1]), "=s"(r.c[2]) : "s"(p));
  }
  return r;
}

template <int NIN, int NOUTF, int NOUT, int ACT, bool STRICT, bool POISON, class T>
__device__ __forceinline__ void linear_chunked(const float* __restrict__ w, const T* x, T* y,
                                               T p0) {
  constexpr int S = Lin<NIN, NOUTF>::stride;
  const auto wc = sload<Lin<NIN, NOUTF>::floats / 16>(w);
#pragma unroll
  for (int o = 0; o < NOUT; ++o) {
    T a = splat(wc[NOUTF * S + o], T{});
    if constexpr (POISON) a += p0;
#pragma unroll
    for (int k = 0; k < NIN; ++k) a = fmaT(wc[o * S + k], x[k], a);
    y[o] = act<ACT, STRICT>(a);
  }
}

// Linear through the chunked scalar path when the block fits 3 chunks.
template <int NIN, int NOUTF, int NOUT, int ACT, bool STRICT, bool POISON, bool CH, class T,
          class WP>
__device__ __forceinline__ void linear_any(const WP* __restrict__ w, const T* x, T* y, T p0) {
  if constexpr (CH && sizeof(WP) == 4 && Lin<NIN, NOUTF>::floats <= 48)
    linear_chunked<NIN, NOUTF, NOUT, ACT, STRICT, POISON>(w, x, y, p0);
  else
    linear<NIN, NOUTF, NOUT, ACT, STRICT, POISON>(w, x, y, p0);
}

// Conditioner MLP on the conditioning half c[DC]; HACT: hidden activation.
template <int D, int H1, int H2, int NO, bool STRICT, bool CH = false, int HACT = 1, class T,
          class WP>
__device__ __forceinline__ void mlp(const WP* __restrict__ w, const T* c, T p0, T* o) {
  constexpr int DC = D - D / 2;
  const T z = splat(0.f, T{});
  if constexpr (H1 == 0) {
    linear_any<DC, D, NO, 0, STRICT, STRICT, CH>(w, c, o, p0);
  } else if constexpr (H2 == 0) {
    T h1[H1];
    linear_any<DC, H1, H1, HACT, STRICT, STRICT, CH>(w, c, h1, p0);
    linear_any<H1, D, NO, 0, STRICT, false, CH>(w + Lin<DC, H1>::floats, h1, o, z);
  } else {
    T h1[H1], h2[H2];
    linear_any<DC, H1, H1, HACT, STRICT, STRICT, CH>(w, c, h1, p0);
    const WP* w2 = w + Lin<DC, H1>::floats;
    linear_any<H1, H2, H2, HACT, STRICT, false, CH>(w2, h1, h2, z);
    linear_any<H2, D, NO, 0, STRICT, false, CH>(w2 + Lin<H1, H2>::floats, h2, o, z);
  }
}

// Register holding logical position j in orientation O (O: row stored reversed).
template <int D, bool O>
__device__ __forceinline__ constexpr int R(int j) { return O ? D - 1 - j : j; }

// Opaque copy: keeps LLVM from turning a select chain over an array into a
// dynamically indexed load (which demotes the array to scratch memory).
template <class T>
__device__ __forceinline__ T opaque(T a) {
  asm("" : "+v"(a));
  return a;
}

template <int D, class T>
__device__ __forceinline__ T pick(const T* v, int idx) {
  // opaque(): without it LLVM folds the chain into v[idx] and keeps v in
  // scratch (measured: ~120 B/row of extra HBM writes on cfg2).
  T r = opaque(v[0]);
#pragma unroll
  for (int k = 1; k < D; ++k) r = (idx == k) ? opaque(v[k]) : r;
  return r;
}

// Gather v (orientation O) into orientation !O through the layer's uniform
// index table: new logical j takes old logical q[j].
template <int D, bool O, class T>
__device__ __forceinline__ void permute(T* v, const int32_t* __restrict__ q) {
  T nv[D];
#pragma unroll
  for (int j = 0; j < D; ++j) nv[R<D, !O>(j)] = pick<D>(v, R<D, O>(q[j]));
#pragma unroll
  for (int k = 0; k < D; ++k) v[k] = nv[k];
}

// One coupling layer, input in orientation O, output in orientation !O.
// SACT: the s-net's hidden activation (1 ReLU; 2 tanh, legacy CNF_OPT_S_TANH).
template <int D, int H1, int H2, bool INV, bool STRICT, bool O, bool FX, bool CH, int SACT = 1,
          class T, class WP>
__device__ __forceinline__ void step(T* v, T& ld, const WP* __restrict__ wl, int scale,
                                     int shift, int net_floats, bool perm,
                                     const int32_t* __restrict__ q) {
  constexpr int DT = D / 2, DC = D - D / 2;
  constexpr int NO = STRICT ? D : DT;
  const T zero = splat(0.f, T{});
  // Inverse: flip (+rev_perm) BEFORE the coupling (flows/flows.py:115-117).
  constexpr bool OC = INV ? !O : O;  // orientation the coupling sees
  if constexpr (INV) {
    if (perm) permute<D, O>(v, q);
  }
  T c[DC];
#pragma unroll
  for (int k = 0; k < DC; ++k) c[k] = v[R<D, OC>(DT + k)];
  T p0 = zero;
  if constexpr (STRICT) {
    // x_b = mask*x: a non-finite transformed input makes 0*x = NaN feed both nets.
#pragma unroll
    for (int j = 0; j < DT; ++j) p0 += 0.f * v[R<D, OC>(j)];
  }
  T s[NO], t[NO];
  if (scale) {
    mlp<D, H1, H2, NO, STRICT, CH, SACT>(wl, c, p0, s);
    wl += net_floats;
  } else {
#pragma unroll
    for (int j = 0; j < NO; ++j) s[j] = zero;
  }
  if (shift) {
    mlp<D, H1, H2, NO, STRICT, CH>(wl, c, p0, t);
  } else {
#pragma unroll
    for (int j = 0; j < NO; ++j) t[j] = zero;
  }
#pragma unroll
  for (int j = 0; j < DT; ++j) {
    T& x = v[R<D, OC>(j)];
    if constexpr (!INV) {
      T y = fmaV(x, expT<FX>(s[j]), t[j]);
      x = STRICT ? 0.f * x + y : y;
      ld += s[j];
    } else {
      T y = (x - t[j]) * expT<FX>(-s[j]);
      x = STRICT ? 0.f * x + y : y;
      ld -= s[j];
    }
  }
  if constexpr (STRICT) {
    // masked positions: x + 0*(x*exp(s)+t) is NaN when exp(s) overflows.
#pragma unroll
    for (int j = DT; j < D; ++j) {
      T& x = v[R<D, OC>(j)];
      T y = INV ? (x - t[j]) * expT<false>(-s[j]) : fmaV(x, expT<false>(s[j]), t[j]);
      x = x + 0.f * y;
      ld += 0.f * s[j];
    }
  }
  // Forward: flip (+perm) AFTER the coupling (flows/flows.py:110-112).
  if constexpr (!INV) {
    if (perm) permute<D, O>(v, q);
  }
}

// gin[k] = sum_o W[o][k] * gout[o], k < NIN, o < NOUT  (transpose product, compact layout)
template <int NIN, int NOUTF, int NOUT>
__device__ __forceinline__ void linear_t(const float* __restrict__ w, const float* gout,
                                         float* gin) {
  constexpr int S = Lin<NIN, NOUTF>::stride;
#pragma unroll
  for (int k = 0; k < NIN; ++k) {
    float a = 0.f;
#pragma unroll
    for (int o = 0; o < NOUT; ++o) a = fmaf(w[o * S + k], gout[o], a);
    gin[k] = a;
  }
}

}  // namespace valu
}  // namespace cnf
