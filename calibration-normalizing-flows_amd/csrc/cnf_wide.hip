// Wide coupling stacks on the f32 matrix cores with every activation in
// registers (CIFAR-100 logits: D=100, hidden_size=[100,100], L=12 -- the
// MFMA-bound configuration of BASELINE.json, configs[3]).
//
// k_tile (cnf_tile.hip) keeps 16 vectors per wave in LDS and reads one A
// operand from L2 per MFMA, so each weight byte serves 16 rows and the wave
// alternates LDS and L2 waits.  Here:
//   * v_mfma_f32_32x32x2_f32 computes Y^T = W . X^T for 32 rows per wave
//     (M = output features, N = rows, K = input features): every weight byte
//     serves 32 rows;
//   * a Linear's 32x32 accumulator tile IS the next Linear's B operand: lane
//     l holds row l&31 and, in register r, feature
//         slot(mt, r, h) = 32 mt + (r & 3) + 8 (r >> 2) + 4 h,   h = l >> 5,
//     which is exactly the B layout of a K-step (lane half h supplies k = h).
//     cnf_prepare lays the A tiles out in that K order, so a conditioner MLP
//     runs register to register; the bias is a first K-step against a ones
//     operand;
//   * the nets always see the conditioning half at slots [DT, D) and write s, t
//     over [0, DT) (the mask of flows/flows.py:81-86); each layer's flip and
//     random permutation (flows/flows.py:110-117) is one per-wave LDS gather
//     through the layer's index table (~200 LDS operations beside ~870 MFMAs);
//   * only K-steps that hold a real input and only M-tiles that hold a real
//     output are issued (compile-time lists): 74 % of the issued MACs are the
//     reference's at D=100.
// f32 in / f32 accumulate is an exact fmaf chain (cdna_hip_programming.md,
// FP32-input MFMA): the precision of the reference's fp32 addmm.
//
// The shipped library serves these shapes with k_wide16 (cnf_wide16.hip,
// 16x16x4 tiles: 1.17x the reference's MACs instead of 1.39x, 0.72 of the
// MFMA roof); this 32x32x2 family is compiled only into A/B builds
// (make ab ABSRC=cnf_wide DEFS=-DCNF_WIDE16=0).  The shape table and the
// wide_* dispatchers below are shared.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <utility>

#include "cnf_internal.h"

// CNF_WIDE16 (default 1): the wide_* entry points run k_wide16 (16x16x4
// tiles, cnf_wide16.hip) for every shape of the table; 0 compiles and runs
// k_wide's 32x32x2 tiles instead (A/B builds only).
#ifndef CNF_WIDE16
#define CNF_WIDE16 1
#endif

namespace cnf {
namespace {

// the shapes the register-MFMA family serves: CIFAR-100 flows (cfg4, and its
// one- / no-hidden-layer variants) and the mid-width fixture shape
struct WShape {
  int D, H1, H2;
};
constexpr WShape kWShapes[] = {{100, 100, 100}, {100, 100, 0}, {100, 0, 0}, {32, 64, 64}};

bool wshape(const Shape& s) {
  if (s.n_lin > 3) return false;
  const int h1 = s.n_lin >= 2 ? s.units[1] : 0, h2 = s.n_lin >= 3 ? s.units[2] : 0;
  for (const WShape& e : kWShapes)
    if (e.D == s.D && e.H1 == h1 && e.H2 == h2) return true;
  return false;
}

#if !CNF_WIDE16

typedef float v16 __attribute__((ext_vector_type(16)));

#ifndef CNF_WIDE_SB
#define CNF_WIDE_SB 0  // sched_barrier mask: what may cross a K-step boundary
#endif
#ifndef CNF_WIDE_WPE
#define CNF_WIDE_WPE 2  // waves per SIMD
#endif
#ifndef CNF_WIDE_PMAX
#define CNF_WIDE_PMAX (CNF_WIDE_WPE == 1 ? 32 : 16)  // deepest A-operand ring
#endif

constexpr int kWRows = 32;  // rows per wave
constexpr int kWWaves = 4;  // waves per block

__host__ __device__ constexpr int slot_of(int mt, int r, int h) {
  return 32 * mt + (r & 3) + 8 * (r >> 2) + 4 * h;
}

// Compile-time geometry of one conditioner MLP (H = 0: absent hidden layer).
template <int D, int H1, int H2>
struct WG {
  static constexpr int DT = D / 2;
  static constexpr int NL = H1 == 0 ? 1 : (H2 == 0 ? 2 : 3);
  static constexpr int TX = (D + 31) / 32;
  static constexpr int hid(int i) { return i == 1 ? H1 : H2; }
  // Linear i reads the state (K over the conditioning half) or a hidden layer
  static constexpr int tin(int i) { return i == 0 ? TX : (hid(i) + 31) / 32; }
  static constexpr int tout(int i) {
    return i == NL - 1 ? (DT + 31) / 32 : (hid(i + 1) + 31) / 32;
  }
  static constexpr bool kact(int i, int mt, int r) {
    for (int h = 0; h < 2; ++h) {
      const int s = slot_of(mt, r, h);
      if (i == 0 ? (s >= DT && s < D) : (s < hid(i))) return true;
    }
    return false;
  }
  // K-steps: 0 = bias (ones operand), then every active (mt, r): code mt*16 + r
  static constexpr int nks(int i) {
    int n = 1;
    for (int mt = 0; mt < tin(i); ++mt)
      for (int r = 0; r < 16; ++r) n += kact(i, mt, r) ? 1 : 0;
    return n;
  }
  static constexpr int code(int i, int n) {
    if (n == 0) return -1;
    int c = 0;
    for (int mt = 0; mt < tin(i); ++mt)
      for (int r = 0; r < 16; ++r)
        if (kact(i, mt, r) && ++c == n) return mt * 16 + r;
    return -2;
  }
  static constexpr int lin_floats(int i) { return tout(i) * nks(i) * 64; }
  static constexpr int lin_off(int i) { return i == 0 ? 0 : lin_off(i - 1) + lin_floats(i - 1); }
  static constexpr int NF = lin_off(NL);  // floats per net
  static constexpr int TS = tout(NL - 1);  // s / t tiles
  static constexpr int TH1 = H1 > 0 ? (H1 + 31) / 32 : 1, TH2 = H2 > 0 ? (H2 + 31) / 32 : 1;
  static constexpr int sbefore(int i) { return i == 0 ? 0 : sbefore(i - 1) + tout(i - 1) * nks(i - 1); }
  static constexpr int mfmas() { return sbefore(NL); }  // K-steps (= MFMAs) per net
};

// A-operand ring depth for a layer of LS K-steps: the ring runs on across
// layers (the next layer's first steps are fetched during this layer's last),
// so its depth must divide LS; the deepest divisor in [6, pmax].
__host__ __device__ constexpr int ring_depth(int ls, int pmax) {
  for (int p = pmax; p >= 6; --p)
    if (ls % p == 0) return p;
  return 1;
}

__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// K-step N of M-tile MT of Linear I of net NET: A from the prefetch ring,
// which is refilled P steps ahead along the layer's flat A stream (both nets,
// every Linear, 64 floats per step) and on into the next layer's (wn).
template <class G, int NETS, int NET, int I, int MT, int N, int P, int TIN>
__device__ __forceinline__ void kstep(v16& acc, float (&ring)[P], const float* __restrict__ a,
                                      const float* __restrict__ an, const v16 (&in)[TIN],
                                      float ones) {
  constexpr int LS = NETS * G::mfmas();
  constexpr int T = NET * G::mfmas() + G::sbefore(I) + MT * G::nks(I) + N;
  const float av = ring[T % P];
  if constexpr (T + P < LS) ring[T % P] = a[(T + P) * 64];
  else ring[T % P] = an[(T + P - LS) * 64];
  constexpr int C = G::code(I, N);
  float bv;
  if constexpr (C < 0) bv = ones;
  else bv = in[C >> 4][C & 15];
  acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
  // keep each refill where it is: left alone, the scheduler sinks the loads
  // next to their use and every MFMA waits vmcnt(0)
  __builtin_amdgcn_sched_barrier(CNF_WIDE_SB);
}

// Epilogues of an M-tile's accumulator: store (hidden layers with ReLU, or
// the t-net's output) or the fused affine update of the state (the s-net's
// last Linear, run after the t-net: each s tile is applied and dropped, so s
// and t are never live together).
template <bool RELU, int TOUT>
struct EpOut {
  v16 (&o)[TOUT];
  template <int MT>
  __device__ __forceinline__ void put(v16 acc) {
    if constexpr (RELU) {
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = fmaxf(acc[r], 0.f);
    }
    o[MT] = acc;
  }
};

template <bool INV, int TX, int TS>
struct EpAffine {
  v16 (&X)[TX];
  const v16 (&T)[TS];
  float& ld;
  template <int MT>
  __device__ __forceinline__ void put(v16 s) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      // slots >= DT of these tiles got s = t = 0 (zero A rows and bias): x stays x
      // exp(s) = 2^(s log2 e): one v_exp_f32 (|rel err| < 1e-6 for |s| < 10)
      const float e = __builtin_amdgcn_exp2f((INV ? -s[r] : s[r]) * 1.4426950408889634f);
      const float x = X[MT][r];
      X[MT][r] = INV ? (x - T[MT][r]) * e : fmaf(x, e, T[MT][r]);
      ld += INV ? -s[r] : s[r];
    }
  }
};

template <class G, int NETS, int NET, int I, int MT, int P, int TIN, class EP, int... N>
__device__ __forceinline__ void mtile(float (&ring)[P], const float* __restrict__ a,
                                      const float* __restrict__ an, const v16 (&in)[TIN],
                                      EP& ep, float ones, std::integer_sequence<int, N...>) {
  v16 acc = {};
  (kstep<G, NETS, NET, I, MT, N, P>(acc, ring, a, an, in, ones), ...);
  ep.template put<MT>(acc);
}

template <class G, int NETS, int NET, int I, int P, int TIN, class EP, int... M>
__device__ __forceinline__ void lin(float (&ring)[P], const float* __restrict__ a,
                                    const float* __restrict__ an, const v16 (&in)[TIN],
                                    EP& ep, float ones, std::integer_sequence<int, M...>) {
  (mtile<G, NETS, NET, I, M>(ring, a, an, in, ep, ones,
                             std::make_integer_sequence<int, G::nks(I)>{}), ...);
}

// One conditioner MLP (stream position NET of the layer) on the state X; its
// last Linear's tiles go to ep.  a / an: this layer's and the next layer's A
// streams.
template <class G, int NETS, int NET, int P, class EP>
__device__ __forceinline__ void net(float (&ring)[P], const float* __restrict__ a,
                                    const float* __restrict__ an, const v16 (&X)[G::TX], EP& ep,
                                    float ones) {
  using MS0 = std::make_integer_sequence<int, G::tout(0)>;
  if constexpr (G::NL == 1) {
    lin<G, NETS, NET, 0>(ring, a, an, X, ep, ones, MS0{});
  } else if constexpr (G::NL == 2) {
    v16 h1[G::TH1];
    EpOut<true, G::TH1> e1{h1};
    lin<G, NETS, NET, 0>(ring, a, an, X, e1, ones, MS0{});
    lin<G, NETS, NET, 1>(ring, a, an, h1, ep, ones, std::make_integer_sequence<int, G::tout(1)>{});
  } else {
    v16 h1[G::TH1], h2[G::TH2];
    EpOut<true, G::TH1> e1{h1};
    EpOut<true, G::TH2> e2{h2};
    lin<G, NETS, NET, 0>(ring, a, an, X, e1, ones, MS0{});
    lin<G, NETS, NET, 1>(ring, a, an, h1, e2, ones, std::make_integer_sequence<int, G::tout(1)>{});
    lin<G, NETS, NET, 2>(ring, a, an, h2, ep, ones, std::make_integer_sequence<int, G::tout(2)>{});
  }
}

// X slots -> LDS rows [row][slot] (slot < D)
template <int D, int TX>
__device__ __forceinline__ void put_state(float* st, int S, const v16 (&X)[TX], int lane) {
  const int row = lane & 31, h = lane >> 5;
#pragma unroll
  for (int mt = 0; mt < TX; ++mt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int s = slot_of(mt, r, h);
      if (s < D) st[row * S + s] = X[mt][r];
    }
}

// New state: slot j takes old logical q[j] (the layer's table, staged in LDS)
template <int D, int TX>
__device__ __forceinline__ void relayout(float* st, int* qs, int S, const int32_t* __restrict__ q,
                                         v16 (&X)[TX], int lane) {
  for (int j = lane; j < D; j += 64) qs[j] = q[j];
  put_state<D, TX>(st, S, X, lane);
  wsync();
  const int row = lane & 31, h = lane >> 5;
#pragma unroll
  for (int mt = 0; mt < TX; ++mt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int s = slot_of(mt, r, h);
      X[mt][r] = s < D ? st[row * S + qs[s]] : 0.f;
    }
  wsync();
}

// The calibrator's predict on rows staged in LDS (calibrators.py:40-44,
// 330-353): two lanes per row (lane l: row l & 31, features of half l >> 5),
// their partial sums / maxima joined by one cross-half shuffle.
template <int D>
__device__ __forceinline__ void row_centre(float* st, int S, int lane) {
  constexpr int HF = (D + 1) / 2;
  const int row = lane & 31, f0 = (lane >> 5) * HF, f1 = f0 + HF < D ? f0 + HF : D;
  float* r = st + row * S;
  float s = 0.f;
  for (int f = f0; f < f1; ++f) s += r[f];
  s += __shfl_xor(s, 32);
  const float mu = s * (1.f / D);
  for (int f = f0; f < f1; ++f) r[f] -= mu;
}
// softmax(log(softmax(z) + 1e-7) - log_priors), in place
template <int D>
__device__ __forceinline__ void row_predict(float* st, int S, int lane,
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

// PRED: the fused calibrated predict (centre, forward, softmax, prior
// correction; lpri = log priors [D]), else forward (INV false) / inverse.
template <int D, int H1, int H2, bool INV, int NETS, bool PRED = false>
__global__ __launch_bounds__(64 * kWWaves, CNF_WIDE_WPE) void k_wide(
    const float* __restrict__ W, const int32_t* __restrict__ qtab,
    const float* __restrict__ in, float* __restrict__ out, float* __restrict__ ld_out,
    int64_t B, int L, const float* __restrict__ lpri) {
  using G = WG<D, H1, H2>;
  constexpr int TX = G::TX, TS = G::TS;
  constexpr int S = D | 1;  // odd LDS row stride: one slot of 32 rows spans 32 banks
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t row0 = ((int64_t)blockIdx.x * kWWaves + wave) * kWRows;
  if (row0 >= B) return;  // waves synchronise only with themselves
  const int nrows = (int)((B - row0) < kWRows ? (B - row0) : kWRows);
  float* st = smem + wave * (kWRows * S + D);
  int* qs = reinterpret_cast<int*>(st + kWRows * S);
  const float ones = lane < 32 ? 1.f : 0.f;

  // rows -> LDS (coalesced) -> slots
  const float* src = in + row0 * D;
  for (int i = lane; i < kWRows * D; i += 64) {
    const int r = i / D, f = i - r * D;
    st[r * S + f] = r < nrows ? src[i] : 0.f;
  }
  wsync();
  if constexpr (PRED) {  // x - mean(x) per row (calibrators.py:42)
    row_centre<D>(st, S, lane);
    wsync();
  }
  v16 X[TX];
  {
    const int row = lane & 31, h = lane >> 5;
#pragma unroll
    for (int mt = 0; mt < TX; ++mt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int s = slot_of(mt, r, h);
        X[mt][r] = s < D ? st[row * S + s] : 0.f;
      }
  }
  wsync();

  // the A stream: one ring for the whole launch, P K-steps ahead of the MFMAs
  constexpr int P = ring_depth(NETS * G::mfmas(), CNF_WIDE_PMAX);
  float ring[P];
  {
    const float* a0 = W + (int64_t)(INV ? L - 1 : 0) * NETS * G::NF + lane;
#pragma unroll
    for (int j = 0; j < P; ++j) ring[j] = a0[j * 64];
  }
  float ld = 0.f;
  for (int stp = 0; stp < L; ++stp) {
    const int l = INV ? L - 1 - stp : stp;
    const int ln = stp + 1 < L ? (INV ? l - 1 : l + 1) : l;  // last layer: harmless re-read
    const int32_t* __restrict__ q = qtab + l * D;
    if constexpr (INV) relayout<D, TX>(st, qs, S, q, X, lane);  // flip / rev_perm first
    const float* __restrict__ wl = W + (int64_t)l * NETS * G::NF + lane;
    const float* __restrict__ wn = W + (int64_t)ln * NETS * G::NF + lane;
    v16 Tv[TS];
    EpOut<false, TS> et{Tv};
    if constexpr (NETS == 2) {  // stream order (cnf_prepare): t-net, then s-net
      net<G, 2, 0>(ring, wl, wn, X, et, ones);
      EpAffine<INV, TX, TS> ea{X, Tv, ld};
      net<G, 2, 1>(ring, wl, wn, X, ea, ones);
    } else {
      net<G, 1, 0>(ring, wl, wn, X, et, ones);
#pragma unroll
      for (int mt = 0; mt < TS; ++mt)
#pragma unroll
        for (int r = 0; r < 16; ++r) X[mt][r] = INV ? X[mt][r] - Tv[mt][r] : X[mt][r] + Tv[mt][r];
    }
    if constexpr (!INV) relayout<D, TX>(st, qs, S, q, X, lane);  // perm then flip
  }

  // slots -> LDS rows -> coalesced stores
  put_state<D, TX>(st, S, X, lane);
  wsync();
  if constexpr (PRED) {
    row_predict<D>(st, S, lane, lpri);
    wsync();
  }
  if (out) {
    float* dst = out + row0 * D;
    for (int i = lane; i < nrows * D; i += 64) {
      const int r = i / D, f = i - r * D;
      dst[i] = st[r * S + f];
    }
  }
  ld += __shfl_xor(ld, 32);
  if (ld_out && lane < nrows) ld_out[row0 + lane] = ld;
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
using WFn = void (*)(const float*, const int32_t*, const float*, float*, float*, int64_t, int,
                    const float*);

constexpr int kMaxKs = 1 + (CNF_MAX_WIDTH / 32 + 1) * 16;  // bias + widest input x 16

// One Linear's A-tile recipe for the prepare kernel.
struct WSeg {
  const float* W;
  const float* b;
  int64_t dst;              // float offset in the wide region
  int nm, nk;               // M-tiles, K-steps (incl. the bias step)
  int first, last;          // K over the state's conditioning half / M over s, t slots
  int nin_full, nout_full;  // the reference weight is [nout_full][nin_full]
  int nin_real;             // hidden input width (first: D)
  int D, DT;
  int16_t code[kMaxKs];     // K-step codes: -1 bias, mt*16 + r
};

struct WPrepArgs {
  WSeg seg[6];  // 2 nets x up to 3 Linears
  int nseg;
};

__global__ void k_prepare_wide(WPrepArgs a, float* __restrict__ wreg) {
  const WSeg& g = a.seg[blockIdx.x];
  float* dst = wreg + g.dst;
  const int64_t n = (int64_t)g.nm * g.nk * 64;
  for (int64_t e = threadIdx.x; e < n; e += blockDim.x) {
    const int lane = (int)(e & 63), ks = (int)((e >> 6) % g.nk), mt = (int)((e >> 6) / g.nk);
    const int i = lane & 31, h = lane >> 5;
    const int m = 32 * mt + i;  // M index: output slot (last) or hidden unit
    const int o = g.last ? (m < g.DT ? m : -1) : (m < g.nout_full ? m : -1);
    float v = 0.f;
    if (o >= 0) {
      const int c = g.code[ks];
      if (c < 0) {
        v = h == 0 ? g.b[o] : 0.f;
      } else {
        const int s = slot_of(c >> 4, c & 15, h);
        // first Linear sees the masked state: only the conditioning half is live
        const bool ok = g.first ? (s >= g.DT && s < g.D) : (s < g.nin_real);
        if (ok) v = g.W[(int64_t)o * g.nin_full + s];
      }
    }
    dst[e] = v;
  }
}

template <int D, int H1, int H2>
void fill_segment(int i, WSeg* g) {
  using Gm = WG<D, H1, H2>;
  g->nm = Gm::tout(i);
  g->nk = Gm::nks(i);
  g->first = i == 0;
  g->last = i == Gm::NL - 1;
  g->D = D;
  g->DT = Gm::DT;
  g->nin_real = i == 0 ? D : Gm::hid(i);
  for (int n = 0; n < g->nk && n < kMaxKs; ++n) g->code[n] = (int16_t)Gm::code(i, n);
}

struct WEntry {
  int D, H1, H2;
  WFn fn[2][3];  // [nets - 1][forward, inverse, predict]
  int net_floats, lin_off[3], mfmas;
  void (*fill)(int, WSeg*);
};

#define CNF_WG(D, H1, H2) WG<D, H1, H2>
#define CNF_WIDE(D, H1, H2)                                                       \
  {D, H1, H2,                                                                     \
   {{k_wide<D, H1, H2, false, 1>, k_wide<D, H1, H2, true, 1>,                     \
     k_wide<D, H1, H2, false, 1, true>},                                          \
    {k_wide<D, H1, H2, false, 2>, k_wide<D, H1, H2, true, 2>,                     \
     k_wide<D, H1, H2, false, 2, true>}},                                         \
   CNF_WG(D, H1, H2)::NF,                                                         \
   {0, CNF_WG(D, H1, H2)::lin_off(1), CNF_WG(D, H1, H2)::lin_off(2)},             \
   CNF_WG(D, H1, H2)::mfmas(), fill_segment<D, H1, H2>}

// the kernels of every shape of kWShapes
const WEntry kWTable[] = {
    CNF_WIDE(100, 100, 100),
    CNF_WIDE(100, 100, 0),
    CNF_WIDE(100, 0, 0),
    CNF_WIDE(32, 64, 64),
};

const WEntry* wfind(const Shape& s) {
  if (s.n_lin > 3) return nullptr;
  const int h1 = s.n_lin >= 2 ? s.units[1] : 0, h2 = s.n_lin >= 3 ? s.units[2] : 0;
  for (const WEntry& e : kWTable)
    if (e.D == s.D && e.H1 == h1 && e.H2 == h2) return &e;
  return nullptr;
}

size_t wide_lds(const Shape& s) { return (size_t)kWWaves * (kWRows * (s.D | 1) + s.D) * 4; }

#endif  // !CNF_WIDE16

}  // namespace

int64_t wide_layer_floats(const Shape& s) {
#if CNF_WIDE16
  return wshape(s) ? wide16_layer_floats(s) : 0;
#else
  const WEntry* e = wfind(s);
  return e ? (int64_t)e->net_floats * s.nets : 0;
#endif
}

// Final-output forward / inverse of shift-on, non-strict stacks in the table;
// every-layer outputs and strict_nan stay on k_tile.
bool wide_ok(const Shape& s) {
  return wshape(s) && s.shift && !s.strict && !s.alt_mask && !s.s_tanh &&
         !(s.options & CNF_OPT_NO_WIDE);
}

bool wide16_train_ok(const Shape& s) { return CNF_WIDE16 && wide_ok(s); }

int wide_prepare(const Shape& s, const float* const* params, void* prepared, hipStream_t st) {
#if CNF_WIDE16
  return wshape(s) ? wide16_prepare(s, params, prepared, st) : CNF_OK;
#else
  const WEntry* e = wfind(s);
  if (!e) return CNF_OK;
  float* region = reinterpret_cast<float*>(static_cast<char*>(prepared) + idx_bytes(s)) +
                  s.wide_region;
  int pi = 0;
  for (int l = 0; l < s.L; ++l) {
    WPrepArgs a{};
    a.nseg = 0;
    for (int net = 0; net < s.nets; ++net) {
      for (int i = 0; i < s.n_lin; ++i) {
        WSeg& g = a.seg[a.nseg++];
        g.W = params[pi++];
        g.b = params[pi++];
        if (!g.W || !g.b) return CNF_ERR_NULL;
        g.nin_full = s.units[i];
        g.nout_full = s.units[i + 1];
        e->fill(i, &g);
        // stream order: the t-net first (its output must be live when the s-net's
        // last Linear applies the affine update tile by tile)
        const int pos = s.nets == 2 ? 1 - net : net;
        g.dst = ((int64_t)l * s.nets + pos) * e->net_floats + e->lin_off[i];
      }
    }
    hipLaunchKernelGGL(k_prepare_wide, dim3(a.nseg), dim3(256), 0, st, a, region);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
      set_hip_error(err);
      return CNF_ERR_HIP;
    }
  }
  return CNF_OK;
#endif
}

int wide_run(const Shape& s, const void* prepared, const float* in, float* out, float* ld,
             int64_t B, bool inverse, hipStream_t st, const float* log_priors) {
#if CNF_WIDE16
  return wshape(s) ? wide16_run(s, prepared, in, out, ld, B, inverse, st, log_priors)
                   : CNF_ERR_UNSUPPORTED;
#else
  const WEntry* e = wfind(s);
  if (!e) return CNF_ERR_UNSUPPORTED;
  const char* base = static_cast<const char*>(prepared);
  const int32_t* fwd_q = reinterpret_cast<const int32_t*>(base);
  const int32_t* inv_q = fwd_q + s.L * s.D;
  const float* W = reinterpret_cast<const float*>(base + idx_bytes(s)) + s.wide_region;
  const int64_t rows_per_block = (int64_t)kWRows * kWWaves;
  const dim3 grid((unsigned)((B + rows_per_block - 1) / rows_per_block)), block(64 * kWWaves);
  if (log_priors && inverse) return CNF_ERR_UNSUPPORTED;
  WFn fn = e->fn[s.nets - 1][log_priors ? 2 : (inverse ? 1 : 0)];
  hipLaunchKernelGGL(fn, grid, block, wide_lds(s), st, W, inverse ? inv_q : fwd_q, in, out, ld, B,
                     s.L, log_priors);
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    set_hip_error(err);
    return CNF_ERR_HIP;
  }
  return CNF_OK;
#endif
}

}  // namespace cnf
