// Fused multi-layer coupling kernel for narrow flows (VALU, one logit vector
// per lane).  Serves the calibration shapes (D = n_classes up to 16, tiny
// conditioner MLPs such as the reference default hidden_size=[5,5],
// flows/flows.py:71): all L layers run in ONE launch with the row held in
// VGPRs, the conditioner weights wave-uniform (scalar loads into SGPRs, so
// every FMA takes an SGPR operand), the mask folded away (the first Linear
// reads only the D-D//2 conditioning columns, the last Linear produces only
// the D//2 transformed outputs), the per-layer flip folded into a static
// register renaming (layers are processed in pairs), and the per-sample
// log-det kept in a register.
//
// Reference semantics restated (paths in the reference repo):
//   MLP.forward                 flows/utils.py:26-31
//   NvpCouplingLayer.forward    flows/flows.py:101-112
//       z = m*x + (1-m)*(x*exp(s) + t);  ld = sum((1-m)*s);  z = z[:,perm]; z.flip(1)
//   NvpCouplingLayer.backward   flows/flows.py:114-126
//       z = z.flip(1); z = z[:,rev_perm]; x = m*z + (1-m)*(z-t)*exp(-s); ld = sum(-(1-m)s)
//   Flow.forward / backward     flows/flows.py:17-37
//
// HBM traffic per row: D*4 bytes in, D*4 out, 4 for the log-det (+ L*D*4 when
// every intermediate z is kept).  Rows are staged through LDS so global loads
// and stores are 16-byte-per-lane coalesced sweeps of the block's tile.
#include <hip/hip_runtime.h>

#include "cnf_internal.h"

namespace cnf {
namespace {

constexpr int kRows = 256;  // rows (= threads) per block

template <bool STRICT>
__device__ __forceinline__ float relu(float a) {
  // torch.relu propagates NaN; v_max_f32 (IEEE maxNum) would drop it.
  if constexpr (STRICT) return a < 0.f ? 0.f : a;
  else return fmaxf(a, 0.f);
}

// y[o] = b[o] (+p0) + sum_k W[o][OFF+k] * x[k],  o < NOUT, W is [NOUTF][NINF].
template <int NINF, int OFF, int NIN, int NOUTF, int NOUT, bool RELU, bool STRICT, bool POISON>
__device__ __forceinline__ void linear(const float* __restrict__ w, const float* x, float* y,
                                       float p0) {
  const float* __restrict__ b = w + NOUTF * NINF;
#pragma unroll
  for (int o = 0; o < NOUT; ++o) {
    float a = b[o];
    if constexpr (POISON) a += p0;
#pragma unroll
    for (int k = 0; k < NIN; ++k) a = fmaf(w[o * NINF + OFF + k], x[k], a);
    y[o] = RELU ? relu<STRICT>(a) : a;
  }
}

template <int D, int H1, int H2>
struct Net {
  static constexpr int DT = D / 2, DC = D - D / 2;
  static constexpr int floats = H1 == 0   ? D * D + D
                                : H2 == 0 ? H1 * D + H1 + D * H1 + D
                                          : H1 * D + H1 + H2 * H1 + H2 + D * H2 + D;
};

// Conditioner MLP on the conditioning half c[DC] (the masked input x_b has
// zeros at the DT transformed positions, so their weight columns drop out).
template <int D, int H1, int H2, int NO, bool STRICT>
__device__ __forceinline__ void mlp(const float* __restrict__ w, const float* c, float p0,
                                    float* o) {
  constexpr int DT = D / 2, DC = D - D / 2;
  if constexpr (H1 == 0) {
    linear<D, DT, DC, D, NO, false, STRICT, STRICT>(w, c, o, p0);
  } else if constexpr (H2 == 0) {
    float h1[H1];
    linear<D, DT, DC, H1, H1, true, STRICT, STRICT>(w, c, h1, p0);
    linear<H1, 0, H1, D, NO, false, STRICT, false>(w + H1 * D + H1, h1, o, 0.f);
  } else {
    float h1[H1], h2[H2];
    linear<D, DT, DC, H1, H1, true, STRICT, STRICT>(w, c, h1, p0);
    const float* w2 = w + H1 * D + H1;
    linear<H1, 0, H1, H2, H2, true, STRICT, false>(w2, h1, h2, 0.f);
    linear<H2, 0, H2, D, NO, false, STRICT, false>(w2 + H2 * H1 + H2, h2, o, 0.f);
  }
}

// Register holding logical position j in orientation O (O: row stored reversed).
template <int D, bool O>
__device__ __forceinline__ constexpr int R(int j) { return O ? D - 1 - j : j; }

template <int D>
__device__ __forceinline__ float pick(const float* v, int idx) {
  float r = v[0];
#pragma unroll
  for (int k = 1; k < D; ++k) r = (idx == k) ? v[k] : r;
  return r;
}

// Gather v (orientation O) into orientation !O through the layer's uniform
// index table: new logical j takes old logical q[j].
template <int D, bool O>
__device__ __forceinline__ void permute(float* v, const int32_t* __restrict__ q) {
  float nv[D];
#pragma unroll
  for (int j = 0; j < D; ++j) nv[R<D, !O>(j)] = pick<D>(v, R<D, O>(q[j]));
#pragma unroll
  for (int k = 0; k < D; ++k) v[k] = nv[k];
}

// One coupling layer, input in orientation O, output in orientation !O.
template <int D, int H1, int H2, bool INV, bool STRICT, bool O>
__device__ __forceinline__ void step(float* v, float& ld, const float* __restrict__ wl,
                                     int scale, int shift, int net_floats, bool perm,
                                     const int32_t* __restrict__ q) {
  constexpr int DT = D / 2, DC = D - D / 2;
  constexpr int NO = STRICT ? D : DT;
  // Inverse: flip (+rev_perm) BEFORE the coupling (flows/flows.py:115-117).
  constexpr bool OC = INV ? !O : O;  // orientation the coupling sees
  if constexpr (INV) {
    if (perm) permute<D, O>(v, q);
  }
  float c[DC];
#pragma unroll
  for (int k = 0; k < DC; ++k) c[k] = v[R<D, OC>(DT + k)];
  float p0 = 0.f;
  if constexpr (STRICT) {
    // x_b = mask*x: a non-finite transformed input makes 0*x = NaN feed both nets.
#pragma unroll
    for (int j = 0; j < DT; ++j) p0 += 0.f * v[R<D, OC>(j)];
  }
  float s[NO], t[NO];
  if (scale) {
    mlp<D, H1, H2, NO, STRICT>(wl, c, p0, s);
    wl += net_floats;
  } else {
#pragma unroll
    for (int j = 0; j < NO; ++j) s[j] = 0.f;
  }
  if (shift) {
    mlp<D, H1, H2, NO, STRICT>(wl, c, p0, t);
  } else {
#pragma unroll
    for (int j = 0; j < NO; ++j) t[j] = 0.f;
  }
#pragma unroll
  for (int j = 0; j < DT; ++j) {
    float& x = v[R<D, OC>(j)];
    if constexpr (!INV) {
      float y = fmaf(x, expf(s[j]), t[j]);
      x = STRICT ? 0.f * x + y : y;
      ld += s[j];
    } else {
      float y = (x - t[j]) * expf(-s[j]);
      x = STRICT ? 0.f * x + y : y;
      ld -= s[j];
    }
  }
  if constexpr (STRICT) {
    // masked positions: x + 0*(x*exp(s)+t) is NaN when exp(s) overflows.
#pragma unroll
    for (int j = DT; j < D; ++j) {
      float& x = v[R<D, OC>(j)];
      float y = INV ? (x - t[j]) * expf(-s[j]) : fmaf(x, expf(s[j]), t[j]);
      x = x + 0.f * y;
      ld += 0.f * s[j];
    }
  }
  // Forward: flip (+perm) AFTER the coupling (flows/flows.py:110-112).
  if constexpr (!INV) {
    if (perm) permute<D, O>(v, q);
  }
}

__device__ __forceinline__ void tile_load(float* __restrict__ sm, const float* __restrict__ src,
                                          int n, bool vec) {
  const int tid = threadIdx.x;
  int done = 0;
  if (vec) {
    const int n4 = n >> 2;
    const float4* s4 = reinterpret_cast<const float4*>(src);
    float4* d4 = reinterpret_cast<float4*>(sm);
    for (int i = tid; i < n4; i += kRows) d4[i] = s4[i];
    done = n4 << 2;
  }
  for (int i = done + tid; i < n; i += kRows) sm[i] = src[i];
}

__device__ __forceinline__ void tile_store(float* __restrict__ dst, const float* __restrict__ sm,
                                           int n, bool vec) {
  const int tid = threadIdx.x;
  int done = 0;
  if (vec) {
    const int n4 = n >> 2;
    float4* d4 = reinterpret_cast<float4*>(dst);
    const float4* s4 = reinterpret_cast<const float4*>(sm);
    for (int i = tid; i < n4; i += kRows) d4[i] = s4[i];
    done = n4 << 2;
  }
  for (int i = done + tid; i < n; i += kRows) dst[i] = sm[i];
}

// Write the block's rows (registers in orientation O) to dst through LDS.
template <int D, bool O>
__device__ __forceinline__ void store_rows(float* __restrict__ dst, float* sm, const float* v,
                                           int nrows, bool vec) {
  const int tid = threadIdx.x;
  __syncthreads();  // previous users of sm are done
  if (tid < nrows) {
#pragma unroll
    for (int j = 0; j < D; ++j) sm[tid * D + j] = v[R<D, O>(j)];
  }
  __syncthreads();
  tile_store(dst, sm, nrows * D, vec);
}

template <int D, int H1, int H2, bool INV, bool STRICT>
__global__ __launch_bounds__(kRows) void k_valu(
    const float* __restrict__ W, const int32_t* __restrict__ qtab,
    const int32_t* __restrict__ lflag, const float* __restrict__ in, float* __restrict__ out,
    float* __restrict__ ld_out, float* __restrict__ all, int64_t B, int L, int scale, int shift,
    int any_perm, int vec_io) {
  __shared__ __attribute__((aligned(16))) float sm[kRows * D];
  const int tid = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * kRows;
  const int nrows = (int)((B - row0) < kRows ? (B - row0) : kRows);
  const bool vec = vec_io != 0;
  constexpr int NF = Net<D, H1, H2>::floats;
  const int layer_floats = (scale + shift) * NF;

  tile_load(sm, in + row0 * D, nrows * D, vec);
  __syncthreads();
  float v[D];
#pragma unroll
  for (int k = 0; k < D; ++k) v[k] = tid < nrows ? sm[tid * D + k] : 0.f;

  float ld = 0.f;
  // step index i = 0..L-1; layer = i (forward) or L-1-i (inverse)
  auto layer_of = [&](int i) { return INV ? L - 1 - i : i; };
  int i = 0;
  for (; i + 1 < L; i += 2) {
    int la = layer_of(i), lb = layer_of(i + 1);
    bool pa = any_perm && (lflag[la] & kFlagPerm), pb = any_perm && (lflag[lb] & kFlagPerm);
    step<D, H1, H2, INV, STRICT, false>(v, ld, W + (int64_t)la * layer_floats, scale, shift, NF,
                                        pa, qtab + la * D);
    if (all) store_rows<D, true>(all + (int64_t)i * B * D + row0 * D, sm, v, nrows, vec);
    step<D, H1, H2, INV, STRICT, true>(v, ld, W + (int64_t)lb * layer_floats, scale, shift, NF,
                                       pb, qtab + lb * D);
    if (all) store_rows<D, false>(all + (int64_t)(i + 1) * B * D + row0 * D, sm, v, nrows, vec);
  }
  bool odd = i < L;
  if (odd) {
    int la = layer_of(i);
    bool pa = any_perm && (lflag[la] & kFlagPerm);
    step<D, H1, H2, INV, STRICT, false>(v, ld, W + (int64_t)la * layer_floats, scale, shift, NF,
                                        pa, qtab + la * D);
    if (all) store_rows<D, true>(all + (int64_t)i * B * D + row0 * D, sm, v, nrows, vec);
  }
  if (out) {
    if (odd) store_rows<D, true>(out + row0 * D, sm, v, nrows, vec);
    else store_rows<D, false>(out + row0 * D, sm, v, nrows, vec);
  }
  if (ld_out && tid < nrows) ld_out[row0 + tid] = ld;
}

// ---------------------------------------------------------------------------
// instantiation table
// ---------------------------------------------------------------------------
using KFn = void (*)(const float*, const int32_t*, const int32_t*, const float*, float*, float*,
                     float*, int64_t, int, int, int, int, int);

struct Entry {
  int D, H1, H2;
  KFn fn[2][2];  // [inverse][strict]
};

#define CNF_VALU(D, H1, H2)                                                             \
  {D, H1, H2,                                                                           \
   {{k_valu<D, H1, H2, false, false>, k_valu<D, H1, H2, false, true>},                  \
    {k_valu<D, H1, H2, true, false>, k_valu<D, H1, H2, true, true>}}}

const Entry kTable[] = {
    // reference default conditioner hidden_size=[5,5] (flows/flows.py:71)
    CNF_VALU(2, 5, 5), CNF_VALU(3, 5, 5), CNF_VALU(4, 5, 5), CNF_VALU(5, 5, 5),
    CNF_VALU(6, 5, 5), CNF_VALU(8, 5, 5), CNF_VALU(10, 5, 5),
    // notebook settings (hidden_size=[3,3], simulated-predictions-flows.ipynb)
    CNF_VALU(3, 3, 3), CNF_VALU(8, 3, 3), CNF_VALU(10, 3, 3),
    // hidden = [dim] / [dim, dim] (code-old/realNVP.py:47-52 default hidden=[dim])
    CNF_VALU(3, 3, 0), CNF_VALU(10, 10, 0), CNF_VALU(10, 10, 10),
    // single linear (hidden_size=[])
    CNF_VALU(3, 0, 0), CNF_VALU(10, 0, 0),
    CNF_VALU(10, 7, 0), CNF_VALU(10, 5, 0), CNF_VALU(3, 5, 0),
};

}  // namespace

int valu_supported(const Shape& s) {
  int h1 = s.n_lin >= 2 ? s.units[1] : 0;
  int h2 = s.n_lin >= 3 ? s.units[2] : 0;
  if (s.n_lin > 3) return -1;
  for (int i = 0; i < (int)(sizeof(kTable) / sizeof(kTable[0])); ++i)
    if (kTable[i].D == s.D && kTable[i].H1 == h1 && kTable[i].H2 == h2) return i;
  return -1;
}

int valu_run(const Shape& s, const void* prepared, const float* in, float* out, float* ld,
             float* all, int64_t B, bool inverse, hipStream_t st) {
  if (s.valu_id < 0) return CNF_ERR_UNSUPPORTED;
  if (B == 0) return CNF_OK;
  const Entry& e = kTable[s.valu_id];
  const char* base = static_cast<const char*>(prepared);
  const int32_t* fwd_q = reinterpret_cast<const int32_t*>(base);
  const int32_t* inv_q = fwd_q + s.L * s.D;
  const int32_t* flags = inv_q + s.L * s.D;
  const float* W = reinterpret_cast<const float*>(base + idx_bytes(s));
  auto al = [](const void* p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  int vec = al(in) && al(out) && al(all);
  dim3 grid((unsigned)((B + kRows - 1) / kRows)), block(kRows);
  hipLaunchKernelGGL(e.fn[inverse ? 1 : 0][s.strict ? 1 : 0], grid, block, 0, st, W,
                     inverse ? inv_q : fwd_q, flags, in, out, ld, all, B, s.L, s.scale, s.shift,
                     s.any_perm ? 1 : 0, vec);
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    set_hip_error(err);
    return CNF_ERR_HIP;
  }
  return CNF_OK;
}

}  // namespace cnf
