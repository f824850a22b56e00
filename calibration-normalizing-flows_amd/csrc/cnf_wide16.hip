// Wide coupling stacks on 16x16x4 f32 matrix-core tiles with every
// activation in registers: the final-output forward / inverse / predict of
// the CIFAR-100-class flows (D=100, hidden_size=[100,100], L=12: BASELINE.json
// configs[3]).  Replaces k_wide's 32x32x2 tiles (cnf_wide.hip), whose 32-wide
// output tiles and 2-deep K-steps padded a 100-unit layer to 128 outputs.
//
// Reference semantics restated (paths in the reference repo):
//   MLP.forward                 flows/utils.py:26-31
//   NvpCouplingLayer.forward    flows/flows.py:101-112 (and .backward, the
//                               inverse, :114-126)
//   Flow.forward / backward     flows/flows.py:17-37
//   predict                     calibrators.py:40-44, 330-353
//
// Layout.  v_mfma_f32_16x16x4f32 computes Y^T = W . X^T for 16 output units x
// 16 rows x 4 input units; a wave owns 32 rows as two row groups g that share
// every A operand (two MFMAs per weight fragment).  A vector of U units (the
// state's halves, a hidden layer) lives in 16-slot tiles, one v4 per (tile,
// row group): lane l holds slots 16 t + 4 (l >> 4) + q, q = 0..3, of row
// 16 g + (l & 15).  That is the MFMA's C layout AND, register q of tile t, the
// B operand of one K-step (lane group k = l >> 4 supplies slot 16 t + 4 k + q),
// so an accumulator tile feeds the next Linear directly.  Units fill the slots
// q-major -- unit u sits in slot qslot(u) = 16 (u >> 4) + 4 (u & 3) +
// ((u & 15) >> 2) -- so K-step n holds units 4n .. 4n+3 and a U-unit input
// takes ceil(U / 4) steps (100 units: 25, not 28); an output takes ceil(U / 16)
// M-tiles (100: 7 = 112 slots, not 4 x 32 = 128).  Biases initialise the
// accumulators (no bias K-step).  Issued MACs per cfg4 layer: 1.17x the
// reference's, against k_wide's 1.39x.
//
// The state: the conditioning half (features DT..D-1, the masked input the
// nets read, flows/flows.py:81-86) in tiles [0, CS/16), the transformed half
// (features 0..DT-1) in tiles [CS/16, XT); the last Linear's output tile mo is
// the transformed half's tile CS/16 + mo, so the affine update is elementwise
// on registers.  Each layer's flip and random permutation is one per-wave LDS
// gather through the layer's index table.  f32 in / f32 accumulate is an exact
// fmaf chain: the precision of the reference's fp32 addmm.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <utility>

#include "cnf_internal.h"

namespace cnf {
namespace {

typedef float v4 __attribute__((ext_vector_type(4)));

#ifndef CNF_W16_PMAX
#define CNF_W16_PMAX 16  // deepest A-operand ring
#endif

constexpr int kRows = 32;   // rows per wave (two row groups of 16)
constexpr int kWaves = 4;   // waves per block

// the slot of unit u (and, the map being an involution, the unit of slot u)
__host__ __device__ constexpr int qslot(int u) {
  return 16 * (u >> 4) + 4 * (u & 3) + ((u & 15) >> 2);
}
__host__ __device__ constexpr int cdiv(int a, int b) { return (a + b - 1) / b; }

// Compile-time geometry of one conditioner MLP (H = 0: absent hidden layer).
template <int D, int H1, int H2>
struct G16 {
  static constexpr int DT = D / 2, DC = D - D / 2;
  static constexpr int NL = H1 == 0 ? 1 : (H2 == 0 ? 2 : 3);
  static constexpr int CT = cdiv(DC, 16), CS = 16 * CT;  // conditioning tiles / slots
  static constexpr int TT = cdiv(DT, 16);                // transformed tiles
  static constexpr int XT = CT + TT;                      // state tiles
  static constexpr int hid(int i) { return i == 1 ? H1 : H2; }
  static constexpr int nin(int i) { return i == 0 ? DC : hid(i); }
  static constexpr int nout(int i) { return i == NL - 1 ? DT : hid(i + 1); }
  static constexpr int ks(int i) { return cdiv(nin(i), 4); }   // K-steps
  static constexpr int mt(int i) { return cdiv(nout(i), 16); }  // M-tiles
  static constexpr int sbefore(int i) { return i == 0 ? 0 : sbefore(i - 1) + mt(i - 1) * ks(i - 1); }
  static constexpr int steps() { return sbefore(NL); }  // A fragments per net and layer
  static constexpr int bbefore(int i) { return i == 0 ? 0 : bbefore(i - 1) + 16 * mt(i - 1); }
  static constexpr int NA = steps() * 64;  // A-stream floats per net and layer
  static constexpr int NB = bbefore(NL);   // bias floats per net and layer
  static constexpr int T1 = H1 > 0 ? cdiv(H1, 16) : 1, T2 = H2 > 0 ? cdiv(H2, 16) : 1;
};

// feature of state slot s (-1: padding)
template <class G>
__device__ __forceinline__ int feat_of(int s) {
  if (s < G::CS) {
    const int u = qslot(s);
    return u < G::DC ? G::DT + u : -1;
  }
  const int u = qslot(s - G::CS);
  return u < G::DT ? u : -1;
}

// A-operand ring depth: the deepest divisor of the layer's step count in
// [6, pmax] (the ring runs on across layers)
__host__ __device__ constexpr int ring16(int ls, int pmax) {
  for (int p = pmax; p >= 6; --p)
    if (ls % p == 0) return p;
  return 1;
}

__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// K-step N of M-tile MO of Linear I of net NET: A from the prefetch ring,
// refilled P fragments ahead along the layer's A stream (both nets, every
// Linear) and on into the next layer's (an).  Both row groups.
template <class G, int NETS, int NET, int I, int MO, int N, int P, int TIN>
__device__ __forceinline__ void kstep(v4 (&acc)[2], float (&ring)[P], const float* __restrict__ a,
                                      const float* __restrict__ an, const v4 (&in)[TIN][2]) {
  constexpr int LS = NETS * G::steps();
  constexpr int T = NET * G::steps() + G::sbefore(I) + MO * G::ks(I) + N;
  const float av = ring[T % P];
  if constexpr (T + P < LS) ring[T % P] = a[(T + P) * 64];
  else ring[T % P] = an[(T + P - LS) * 64];
  constexpr int t = N >> 2, q = N & 3;
  acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, in[t][0][q], acc[0], 0, 0, 0);
  acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, in[t][1][q], acc[1], 0, 0, 0);
  // keep each refill where it is (left alone, the scheduler sinks the loads
  // next to their use and every MFMA waits for memory)
  __builtin_amdgcn_sched_barrier(0);
}

// Epilogues of an M-tile's accumulators: hidden (ReLU), keep (the t-net's
// output), or the fused affine update of the state (the s-net's last Linear).
template <bool RELU, int TOUT>
struct EpOut {
  v4 (&o)[TOUT][2];
  template <int MO>
  __device__ __forceinline__ void put(v4 (&acc)[2]) {
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      if constexpr (RELU) {
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[g][q] = fmaxf(acc[g][q], 0.f);
      }
      o[MO][g] = acc[g];
    }
  }
};

template <bool INV, int XT, int CT, int TT>
struct EpAffine {
  v4 (&X)[XT][2];
  const v4 (&T)[TT][2];
  float (&ld)[2];
  template <int MO>
  __device__ __forceinline__ void put(v4 (&s)[2]) {
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        // padding slots get s = t = 0 (zero weights and bias): x stays x
        const float sv = s[g][q];
        const float e = __builtin_amdgcn_exp2f((INV ? -sv : sv) * 1.4426950408889634f);
        const float x = X[CT + MO][g][q];
        X[CT + MO][g][q] = INV ? (x - T[MO][g][q]) * e : fmaf(x, e, T[MO][g][q]);
        ld[g] += INV ? -sv : sv;
      }
  }
};

// accumulators of M-tile MO of Linear I start at its biases (the layer's bias
// block: 16 floats per M-tile in slot order)
template <class G, int I, int MO>
__device__ __forceinline__ void bias_init(v4 (&acc)[2], const float* __restrict__ bias, int lane) {
  const float* p = bias + G::bbefore(I) + 16 * MO + 4 * (lane >> 4);
  const v4 b = {p[0], p[1], p[2], p[3]};
  acc[0] = b;
  acc[1] = b;
}

template <class G, int NETS, int NET, int I, int MO, int P, int TIN, class EP, int... N>
__device__ __forceinline__ void mtile(float (&ring)[P], const float* __restrict__ a,
                                      const float* __restrict__ an,
                                      const float* __restrict__ bias, const v4 (&in)[TIN][2],
                                      EP& ep, int lane, std::integer_sequence<int, N...>) {
  v4 acc[2];
  bias_init<G, I, MO>(acc, bias, lane);
  (kstep<G, NETS, NET, I, MO, N, P>(acc, ring, a, an, in), ...);
  ep.template put<MO>(acc);
}

template <class G, int NETS, int NET, int I, int P, int TIN, class EP, int... M>
__device__ __forceinline__ void lin(float (&ring)[P], const float* __restrict__ a,
                                    const float* __restrict__ an, const float* __restrict__ bias,
                                    const v4 (&in)[TIN][2], EP& ep, int lane,
                                    std::integer_sequence<int, M...>) {
  (mtile<G, NETS, NET, I, M>(ring, a, an, bias, in, ep, lane,
                             std::make_integer_sequence<int, G::ks(I)>{}),
   ...);
}

// One conditioner MLP (stream position NET of the layer) on the state's
// conditioning tiles; its last Linear's tiles go to ep.
template <class G, int NETS, int NET, int P, class EP>
__device__ __forceinline__ void net(float (&ring)[P], const float* __restrict__ a,
                                    const float* __restrict__ an, const float* __restrict__ bias,
                                    const v4 (&X)[G::XT][2], EP& ep, int lane) {
  using MS0 = std::make_integer_sequence<int, G::mt(0)>;
  if constexpr (G::NL == 1) {
    lin<G, NETS, NET, 0>(ring, a, an, bias, X, ep, lane, MS0{});
  } else if constexpr (G::NL == 2) {
    v4 h1[G::T1][2];
    EpOut<true, G::T1> e1{h1};
    lin<G, NETS, NET, 0>(ring, a, an, bias, X, e1, lane, MS0{});
    lin<G, NETS, NET, 1>(ring, a, an, bias, h1, ep, lane,
                         std::make_integer_sequence<int, G::mt(1)>{});
  } else {
    v4 h1[G::T1][2], h2[G::T2][2];
    EpOut<true, G::T1> e1{h1};
    EpOut<true, G::T2> e2{h2};
    lin<G, NETS, NET, 0>(ring, a, an, bias, X, e1, lane, MS0{});
    lin<G, NETS, NET, 1>(ring, a, an, bias, h1, e2, lane,
                         std::make_integer_sequence<int, G::mt(1)>{});
    lin<G, NETS, NET, 2>(ring, a, an, bias, h2, ep, lane,
                         std::make_integer_sequence<int, G::mt(2)>{});
  }
}

// state slots -> LDS rows [row][feature]
template <class G>
__device__ __forceinline__ void put_state(float* st, int S, const v4 (&X)[G::XT][2], int lane) {
#pragma unroll
  for (int t = 0; t < G::XT; ++t)
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int f = feat_of<G>(16 * t + 4 * (lane >> 4) + q);
        if (f >= 0) st[(16 * g + (lane & 15)) * S + f] = X[t][g][q];
      }
}

// state slots <- LDS rows through a gather table (slot of feature f takes
// logical q[f]; q == nullptr: identity)
template <class G>
__device__ __forceinline__ void get_state(const float* st, int S, const int* qs, v4 (&X)[G::XT][2],
                                          int lane) {
#pragma unroll
  for (int t = 0; t < G::XT; ++t)
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int f = feat_of<G>(16 * t + 4 * (lane >> 4) + q);
        X[t][g][q] = f >= 0 ? st[(16 * g + (lane & 15)) * S + (qs ? qs[f] : f)] : 0.f;
      }
}

template <class G>
__device__ __forceinline__ void relayout(float* st, int* qs, int S, const int32_t* __restrict__ q,
                                         v4 (&X)[G::XT][2], int lane) {
  for (int j = lane; j < G::DT + G::DC; j += 64) qs[j] = q[j];
  put_state<G>(st, S, X, lane);
  wsync();
  get_state<G>(st, S, qs, X, lane);
  wsync();
}

// the calibrator's predict on LDS rows (calibrators.py:40-44, 330-353)
template <int D>
__device__ __forceinline__ void row_centre16(float* st, int S, int lane) {
  constexpr int HF = (D + 1) / 2;
  const int row = lane & 31, f0 = (lane >> 5) * HF, f1 = f0 + HF < D ? f0 + HF : D;
  float* r = st + row * S;
  float s = 0.f;
  for (int f = f0; f < f1; ++f) s += r[f];
  s += __shfl_xor(s, 32);
  const float mu = s * (1.f / D);
  for (int f = f0; f < f1; ++f) r[f] -= mu;
}
template <int D>
__device__ __forceinline__ void row_predict16(float* st, int S, int lane,
                                              const float* __restrict__ lp) {
  constexpr int HF = (D + 1) / 2;
  constexpr float kL2E = 1.4426950408889634f, kLN2 = 0.6931471805599453f;
  const int row = lane & 31, f0 = (lane >> 5) * HF, f1 = f0 + HF < D ? f0 + HF : D;
  float* r = st + row * S;
  float m = -__builtin_inff();
  for (int f = f0; f < f1; ++f) m = fmaxf(m, r[f]);
  m = fmaxf(m, __shfl_xor(m, 32));
  float se = 0.f;
  for (int f = f0; f < f1; ++f) {
    const float e = __builtin_amdgcn_exp2f((r[f] - m) * kL2E);
    r[f] = e;
    se += e;
  }
  se += __shfl_xor(se, 32);
  const float inv = 1.f / se;
  float m2 = -__builtin_inff();
  for (int f = f0; f < f1; ++f) {
    const float a = __builtin_amdgcn_logf(r[f] * inv + 1e-7f) * kLN2 - lp[f];
    r[f] = a;
    m2 = fmaxf(m2, a);
  }
  m2 = fmaxf(m2, __shfl_xor(m2, 32));
  float s2 = 0.f;
  for (int f = f0; f < f1; ++f) {
    const float e = __builtin_amdgcn_exp2f((r[f] - m2) * kL2E);
    r[f] = e;
    s2 += e;
  }
  s2 += __shfl_xor(s2, 32);
  const float inv2 = 1.f / s2;
  for (int f = f0; f < f1; ++f) r[f] *= inv2;
}

// MODE 0 forward, 1 inverse, 2 predict (centre + forward + calibrated probs)
template <int D, int H1, int H2, int MODE, int NETS>
__global__ __launch_bounds__(64 * kWaves, 2) void k_wide16(
    const float* __restrict__ W, const int32_t* __restrict__ qtab,
    const float* __restrict__ in, float* __restrict__ out, float* __restrict__ ld_out,
    int64_t B, int L, const float* __restrict__ lpri) {
  using G = G16<D, H1, H2>;
  constexpr bool INV = MODE == 1;
  constexpr int XT = G::XT, CT = G::CT, TT = G::TT;
  constexpr int S = D | 1;  // odd LDS row stride
  constexpr int LA = NETS * G::NA, LF = LA + NETS * G::NB;  // A floats / all floats per layer
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t row0 = ((int64_t)blockIdx.x * kWaves + wave) * kRows;
  if (row0 >= B) return;  // waves synchronise only with themselves
  const int nrows = (int)((B - row0) < kRows ? (B - row0) : kRows);
  float* st = smem + wave * (kRows * S + D);
  int* qs = reinterpret_cast<int*>(st + kRows * S);

  // rows -> LDS (coalesced) -> slots
  const float* src = in + row0 * D;
  for (int i = lane; i < kRows * D; i += 64) {
    const int r = i / D, f = i - r * D;
    st[r * S + f] = r < nrows ? src[i] : 0.f;
  }
  wsync();
  if constexpr (MODE == 2) {  // x - mean(x) per row (calibrators.py:42)
    row_centre16<D>(st, S, lane);
    wsync();
  }
  v4 X[XT][2];
  get_state<G>(st, S, nullptr, X, lane);
  wsync();

  // the A stream: one ring for the whole launch, P fragments ahead of the MFMAs
  constexpr int P = ring16(NETS * G::steps(), CNF_W16_PMAX);
  float ring[P];
  {
    const float* a0 = W + (int64_t)(INV ? L - 1 : 0) * LF + lane;
#pragma unroll
    for (int j = 0; j < P; ++j) ring[j] = a0[j * 64];
  }
  float ld[2] = {0.f, 0.f};
  for (int stp = 0; stp < L; ++stp) {
    const int l = INV ? L - 1 - stp : stp;
    const int ln = stp + 1 < L ? (INV ? l - 1 : l + 1) : l;  // last layer: harmless re-read
    const int32_t* __restrict__ q = qtab + l * D;
    if constexpr (INV) relayout<G>(st, qs, S, q, X, lane);  // flip / rev_perm first
    const float* __restrict__ wl = W + (int64_t)l * LF + lane;
    const float* __restrict__ wn = W + (int64_t)ln * LF + lane;
    const float* __restrict__ bl = W + (int64_t)l * LF + LA;  // the layer's bias blocks
    v4 Tv[TT][2];
    EpOut<false, TT> et{Tv};
    if constexpr (NETS == 2) {  // stream order (prepare): t-net, then s-net
      net<G, 2, 0>(ring, wl, wn, bl, X, et, lane);
      EpAffine<INV, XT, CT, TT> ea{X, Tv, ld};
      net<G, 2, 1>(ring, wl, wn, bl + G::NB, X, ea, lane);
    } else {
      net<G, 1, 0>(ring, wl, wn, bl, X, et, lane);
#pragma unroll
      for (int t = 0; t < TT; ++t)
#pragma unroll
        for (int g = 0; g < 2; ++g) X[CT + t][g] = INV ? X[CT + t][g] - Tv[t][g] : X[CT + t][g] + Tv[t][g];
    }
    if constexpr (!INV) relayout<G>(st, qs, S, q, X, lane);  // perm then flip
  }

  // slots -> LDS rows -> coalesced stores
  put_state<G>(st, S, X, lane);
  wsync();
  if constexpr (MODE == 2) {
    row_predict16<D>(st, S, lane, lpri);
    wsync();
  }
  if (out) {
    float* dst = out + row0 * D;
    for (int i = lane; i < nrows * D; i += 64) {
      const int r = i / D, f = i - r * D;
      dst[i] = st[r * S + f];
    }
  }
  // a row's log-det terms are spread over the four lane groups (l >> 4)
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    ld[g] += __shfl_xor(ld[g], 16);
    ld[g] += __shfl_xor(ld[g], 32);
  }
  if (ld_out && lane < 16) {
#pragma unroll
    for (int g = 0; g < 2; ++g)
      if (16 * g + lane < nrows) ld_out[row0 + 16 * g + lane] = ld[g];
  }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
using WFn = void (*)(const float*, const int32_t*, const float*, float*, float*, int64_t, int,
                    const float*);

// One Linear's A / bias recipe for the prepare kernel.
struct WSeg16 {
  const float* W;
  const float* b;
  int64_t adst, bdst;     // float offsets of its A fragments and bias block
  int nm, nk;             // M-tiles, K-steps
  int first;              // input = the conditioning half (weight columns DT..D-1)
  int nin, nout;          // real input / output units
  int nin_full;           // the reference weight is [nout][nin_full]
  int DT;
};
struct WPrep16 {
  WSeg16 seg[6];  // 2 nets x up to 3 Linears
  int nseg;
};

// A fragment (M-tile mo, K-step n), lane l: W[out unit qslot(16 mo + (l & 15))]
// [in unit 4 n + (l >> 4)]; bias block: slot order, zero at padding slots.
__global__ void k_prepare_wide16(WPrep16 a, float* __restrict__ wreg) {
  const WSeg16& g = a.seg[blockIdx.x];
  const int64_t n = (int64_t)g.nm * g.nk * 64;
  for (int64_t e = threadIdx.x; e < n; e += blockDim.x) {
    const int lane = (int)(e & 63), ks = (int)((e >> 6) % g.nk), mo = (int)((e >> 6) / g.nk);
    const int o = qslot(16 * mo + (lane & 15)), u = 4 * ks + (lane >> 4);
    float v = 0.f;
    if (o < g.nout && u < g.nin) v = g.W[(int64_t)o * g.nin_full + (g.first ? g.DT : 0) + u];
    wreg[g.adst + e] = v;
  }
  for (int s = threadIdx.x; s < 16 * g.nm; s += blockDim.x) {
    const int o = qslot(s);
    wreg[g.bdst + s] = o < g.nout ? g.b[o] : 0.f;
  }
}

struct WEntry16 {
  int D, H1, H2;
  WFn fn[2][3];  // [nets - 1][forward, inverse, predict]
  int na, nb;    // A / bias floats per net and layer
  int ks[3], mt[3], abefore[3], bbefore[3];
};

#define CNF_G16(D, H1, H2) G16<D, H1, H2>
#define CNF_W16(D, H1, H2)                                                                    \
  {D, H1, H2,                                                                                 \
   {{k_wide16<D, H1, H2, 0, 1>, k_wide16<D, H1, H2, 1, 1>, k_wide16<D, H1, H2, 2, 1>},        \
    {k_wide16<D, H1, H2, 0, 2>, k_wide16<D, H1, H2, 1, 2>, k_wide16<D, H1, H2, 2, 2>}},       \
   CNF_G16(D, H1, H2)::NA, CNF_G16(D, H1, H2)::NB,                                            \
   {CNF_G16(D, H1, H2)::ks(0), CNF_G16(D, H1, H2)::ks(1), CNF_G16(D, H1, H2)::ks(2)},         \
   {CNF_G16(D, H1, H2)::mt(0), CNF_G16(D, H1, H2)::mt(1), CNF_G16(D, H1, H2)::mt(2)},         \
   {64 * CNF_G16(D, H1, H2)::sbefore(0), 64 * CNF_G16(D, H1, H2)::sbefore(1),                 \
    64 * CNF_G16(D, H1, H2)::sbefore(2)},                                                     \
   {CNF_G16(D, H1, H2)::bbefore(0), CNF_G16(D, H1, H2)::bbefore(1),                           \
    CNF_G16(D, H1, H2)::bbefore(2)}}

const WEntry16 kW16Table[] = {
    CNF_W16(100, 100, 100),
    CNF_W16(100, 100, 0),
    CNF_W16(100, 0, 0),
    CNF_W16(32, 64, 64),
};

const WEntry16* w16find(const Shape& s) {
  if (s.n_lin > 3) return nullptr;
  const int h1 = s.n_lin >= 2 ? s.units[1] : 0, h2 = s.n_lin >= 3 ? s.units[2] : 0;
  for (const WEntry16& e : kW16Table)
    if (e.D == s.D && e.H1 == h1 && e.H2 == h2) return &e;
  return nullptr;
}

size_t w16_lds(const Shape& s) { return (size_t)kWaves * (kRows * (s.D | 1) + s.D) * 4; }

}  // namespace

int64_t wide16_layer_floats(const Shape& s) {
  const WEntry16* e = w16find(s);
  return e ? (int64_t)(e->na + e->nb) * s.nets : 0;
}

int wide16_prepare(const Shape& s, const float* const* params, void* prepared, hipStream_t st) {
  const WEntry16* e = w16find(s);
  if (!e) return CNF_OK;
  float* region = reinterpret_cast<float*>(static_cast<char*>(prepared) + idx_bytes(s)) +
                  s.wide_region;
  const int64_t LA = (int64_t)s.nets * e->na, LF = LA + (int64_t)s.nets * e->nb;
  int pi = 0;
  for (int l = 0; l < s.L; ++l) {
    WPrep16 a{};
    a.nseg = 0;
    for (int net = 0; net < s.nets; ++net) {
      // stream order: the t-net first (its output must be live when the s-net's
      // last Linear applies the affine update tile by tile)
      const int pos = s.nets == 2 ? 1 - net : net;
      for (int i = 0; i < s.n_lin; ++i) {
        WSeg16& g = a.seg[a.nseg++];
        g.W = params[pi++];
        g.b = params[pi++];
        if (!g.W || !g.b) return CNF_ERR_NULL;
        g.nin_full = s.units[i];
        g.first = i == 0;
        g.nin = i == 0 ? s.DC : s.units[i];
        g.nout = i == s.n_lin - 1 ? s.DT : s.units[i + 1];
        g.DT = s.DT;
        g.nm = e->mt[i];
        g.nk = e->ks[i];
        g.adst = (int64_t)l * LF + (int64_t)pos * e->na + e->abefore[i];
        g.bdst = (int64_t)l * LF + LA + (int64_t)pos * e->nb + e->bbefore[i];
      }
    }
    hipLaunchKernelGGL(k_prepare_wide16, dim3(a.nseg), dim3(256), 0, st, a, region);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
      set_hip_error(err);
      return CNF_ERR_HIP;
    }
  }
  return CNF_OK;
}

int wide16_run(const Shape& s, const void* prepared, const float* in, float* out, float* ld,
               int64_t B, bool inverse, hipStream_t st, const float* log_priors) {
  const WEntry16* e = w16find(s);
  if (!e) return CNF_ERR_UNSUPPORTED;
  if (log_priors && inverse) return CNF_ERR_UNSUPPORTED;
  const char* base = static_cast<const char*>(prepared);
  const int32_t* fwd_q = reinterpret_cast<const int32_t*>(base);
  const int32_t* inv_q = fwd_q + s.L * s.D;
  const float* W = reinterpret_cast<const float*>(base + idx_bytes(s)) + s.wide_region;
  const int64_t rows_per_block = (int64_t)kRows * kWaves;
  const dim3 grid((unsigned)((B + rows_per_block - 1) / rows_per_block)), block(64 * kWaves);
  WFn fn = e->fn[s.nets - 1][log_priors ? 2 : (inverse ? 1 : 0)];
  hipLaunchKernelGGL(fn, grid, block, w16_lds(s), st, W, inverse ? inv_q : fwd_q, in, out, ld, B,
                     s.L, log_priors);
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    set_hip_error(err);
    return CNF_ERR_HIP;
  }
  return CNF_OK;
}

}  // namespace cnf
