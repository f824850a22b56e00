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
#include <type_traits>
#include <utility>

#include "cnf_internal.h"

namespace cnf {
namespace {

typedef float v4 __attribute__((ext_vector_type(4)));

#ifndef CNF_W16_PMAX
#define CNF_W16_PMAX 16  // deepest A-operand ring
#endif
#ifndef CNF_W16_FWD_P16
#define CNF_W16_FWD_P16 0  // the same for the forward streams: measured no change (2545 vs 2547 us cfg4 forward), spills the training forward; off
#endif
#ifndef CNF_W16_BWD_P16
#define CNF_W16_BWD_P16 1  // pad the reverse stream per layer to 16-step multiples
#endif

// A-stream layout: 0 fragment-major (step T, lane l at 64 T + l: one dword
// load per lane and K-step); 1 four steps interleaved per lane (steps 4j..4j+3
// of lane l at 256 j + 4 l: one 16-B load per lane every four K-steps)
#ifndef CNF_W16_PACK4
#define CNF_W16_PACK4 1
#endif
#ifndef CNF_W16_REFILL  // packed layout: steps per refill load (4: 16 B, 2: 8 B per lane)
#define CNF_W16_REFILL 4
#endif
constexpr bool kPack4 = CNF_W16_PACK4 != 0;
constexpr int kLaneStride = kPack4 ? 4 : 1;  // a lane's first float of a step group
// float offset (lane 0) of stream step T
__host__ __device__ constexpr int afrag(int T) { return kPack4 ? (T >> 2) * 256 + (T & 3) : T * 64; }

constexpr int kRows = 32;   // rows per wave (two row groups of 16)
constexpr int kWaves = 4;   // waves per block
// row groups per wave of the inference kernel (k_wide16): 2 -> 32 rows per
// wave at 2 waves per SIMD; 4 -> 64 rows per wave at 1 wave per SIMD
#ifndef CNF_W16_RUN_RG
#define CNF_W16_RUN_RG 2
#endif
constexpr int kRunRG = CNF_W16_RUN_RG, kRunRows = 16 * kRunRG;
static_assert(kRunRG == 2 || kRunRG == 4, "CNF_W16_RUN_RG: 2 or 4");

// the slot of unit u (and, the map being an involution, the unit of slot u)
__host__ __device__ constexpr int qslot(int u) {
  return 16 * (u >> 4) + 4 * (u & 3) + ((u & 15) >> 2);
}
__host__ __device__ constexpr int cdiv(int a, int b) { return (a + b - 1) / b; }
// a layer's stream steps with its pads (16-step multiples when p16, 4-step
// multiples for the packed layout)
__host__ __device__ constexpr int pad_ls(int ls, bool p16) {
  return p16 ? cdiv(ls, 16) * 16 : (kPack4 ? cdiv(ls, 4) * 4 : ls);
}
// k_wide16's A stream through LDS (A/B): the block's four waves copy the stream
// by LDS-DMA in chunks of kAC steps (one 1-KiB piece per wave) into two stages,
// and refill their rings from LDS; forward streams padded to 2 kAC steps
#ifndef CNF_W16_LDSA
#define CNF_W16_LDSA 1
#endif
#ifndef CNF_W16_LDSA_CHUNK  // steps per LDS chunk (a multiple of 16: one 1-KiB piece per wave per 16)
#define CNF_W16_LDSA_CHUNK 16
#endif
constexpr int kAC = CNF_W16_LDSA_CHUNK;
#ifndef CNF_W16_LDSA_PMAX  // k_wide16's ring depth with the LDS stream (LDS latency is short)
#define CNF_W16_LDSA_PMAX 8
#endif
__host__ __device__ constexpr int pad_fwd(int ls) {
  return CNF_W16_LDSA ? cdiv(ls, 2 * kAC) * 2 * kAC : pad_ls(ls, CNF_W16_FWD_P16);
}
extern __shared__ __attribute__((aligned(16))) float w16_dyn[];
// the training forward sweep's A stream through LDS as k_wide16's (A/B): its
// chunk waits (vmcnt(0)) also cover the tape stores issued since the last one
#ifndef CNF_W16_TRAIN_LDSA
#define CNF_W16_TRAIN_LDSA 0
#endif

// Compile-time geometry of one conditioner MLP (H = 0: absent hidden layer).
template <int D, int H1, int H2>
struct G16 {
  static constexpr bool kBias = true;  // Linears with biases (the forward)
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
  // A-stream steps per layer: padded to a multiple of 16 (a few fragments no
  // MFMA uses) so the ring can be 16 deep (G16T below)
  template <int NETS>
  static constexpr int lsp() { return pad_fwd(NETS * steps()); }
  static constexpr bool kLdsA = false;
  static constexpr int T1 = H1 > 0 ? cdiv(H1, 16) : 1, T2 = H2 > 0 ? cdiv(H2, 16) : 1;
};
// k_wide16's geometry when its A stream comes through LDS
template <int D, int H1, int H2>
struct G16L : G16<D, H1, H2> {
  static constexpr bool kLdsA = CNF_W16_LDSA != 0;
  // floats of the waves' state areas (the A stages follow)
  static constexpr int kStateFloats = cdiv(kWaves * (kRunRows * (D | 1) + D), 64) * 64;
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
    if (ls % p == 0 && (!kPack4 || p % 4 == 0)) return p;
  return kPack4 ? 4 : 1;
}

// the ring's refill at stream step T (fragment T + P into the slot step T
// just used); packed: every fourth step, the four slots steps T-3..T used
// (a 16-B load per lane)
template <class G, int NETS, int P, int T>
__device__ __forceinline__ void refill(float (&ring)[P], const float* __restrict__ a,
                                       const float* __restrict__ an) {
  constexpr int LS = G::template lsp<NETS>();  // stream steps per layer (pads included)
  if constexpr (G::kLdsA) {
    static_assert(kPack4 && P % 4 == 0 && P <= kAC && LS % (2 * kAC) == 0, "LDS A stream");
    if constexpr ((T & 3) == 3) {
      constexpr int S0 = T - 3 + P;  // first step refilled
      const int lane = threadIdx.x & 63;
      float* stage = w16_dyn + G::kStateFloats;
      if constexpr (S0 % kAC == 0) {
        // chunk S0 / kAC starts: everyone's pieces of it have landed and everyone
        // is done with the chunk before it, whose stage the next chunk takes
        const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        constexpr int S1 = S0 + kAC;  // the next chunk (a = W + layer + 4 lane)
#pragma unroll
        for (int k = 0; k < kAC / 16; ++k) {  // piece k * 4 + w of the chunk's kAC / 4
          const float* src = (S1 < LS ? a + afrag(S1) : an + afrag(S1 - LS)) + 256 * (4 * k + w);
          __builtin_amdgcn_global_load_lds(const_cast<float*>(src),
                                           stage + afrag(S1 % (2 * kAC)) + 256 * (4 * k + w), 16, 0, 0);
        }
      }
      const v4 v = *reinterpret_cast<const v4*>(stage + afrag(S0 % (2 * kAC)) + 4 * lane);
      ring[(T - 3) % P] = v[0];
      ring[(T - 2) % P] = v[1];
      ring[(T - 1) % P] = v[2];
      ring[T % P] = v[3];
    }
  } else if constexpr (!kPack4) {
    if constexpr (T + P < LS) ring[T % P] = a[afrag(T + P)];
    else ring[T % P] = an[afrag(T + P - LS)];
  } else if constexpr (CNF_W16_REFILL == 4 && (T & 3) == 3) {
    static_assert(P % 4 == 0 && LS % 4 == 0, "packed A stream: ring and layer in 4-step groups");
    constexpr int S0 = T - 3 + P;  // first step refilled (a multiple of 4)
    const v4 v = *reinterpret_cast<const v4*>(S0 < LS ? a + afrag(S0) : an + afrag(S0 - LS));
    ring[(T - 3) % P] = v[0];
    ring[(T - 2) % P] = v[1];
    ring[(T - 1) % P] = v[2];
    ring[T % P] = v[3];
  } else if constexpr (CNF_W16_REFILL == 2 && (T & 1) == 1) {
    static_assert(P % 4 == 0 && LS % 4 == 0, "packed A stream: ring and layer in 4-step groups");
    constexpr int S0 = T - 1 + P;  // first step refilled (even)
    typedef float v2 __attribute__((ext_vector_type(2)));
    const v2 v = *reinterpret_cast<const v2*>(S0 < LS ? a + afrag(S0) : an + afrag(S0 - LS));
    ring[(T - 1) % P] = v[0];
    ring[T % P] = v[1];
  }
}


__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// K-step N of M-tile MO of Linear I of net NET: A from the prefetch ring,
// refilled P fragments ahead along the layer's A stream (both nets, every
// Linear) and on into the next layer's (an).  Both row groups.
// The B operand is tile TOFF + N / 4 of `in`.
template <class G, int NETS, int NET, int I, int MO, int N, int TOFF, int P, int TIN, int RG>
__device__ __forceinline__ void kstep(v4 (&acc)[RG], float (&ring)[P], const float* __restrict__ a,
                                      const float* __restrict__ an, const v4 (&in)[TIN][RG]) {
  constexpr int T = NET * G::steps() + G::sbefore(I) + MO * G::ks(I) + N;
  const float av = ring[T % P];
  refill<G, NETS, P, T>(ring, a, an);
  constexpr int t = TOFF + (N >> 2), q = N & 3;
#pragma unroll
  for (int g = 0; g < RG; ++g)
    acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, in[t][g][q], acc[g], 0, 0, 0);
  // keep each refill where it is (left alone, the scheduler sinks the loads
  // next to their use and every MFMA waits for memory)
  __builtin_amdgcn_sched_barrier(0);
}

// the ring's refills for the stream's pad steps (no MFMA)
template <class G, int NETS, int P, int T>
__device__ __forceinline__ void pad_step(float (&ring)[P], const float* __restrict__ a,
                                         const float* __restrict__ an) {
  refill<G, NETS, P, T>(ring, a, an);
  __builtin_amdgcn_sched_barrier(0);
}
template <class G, int NETS, int P, int... K>
__device__ __forceinline__ void pad_steps(float (&ring)[P], const float* __restrict__ a,
                                          const float* __restrict__ an,
                                          std::integer_sequence<int, K...>) {
  (pad_step<G, NETS, P, NETS * G::steps() + K>(ring, a, an), ...);
}

// Epilogues of an M-tile's accumulators: hidden (ReLU), keep (the t-net's
// output), or the fused affine update of the state (the s-net's last Linear).
// pre<MO>() runs before M-tile MO's K-steps (operand prefetch), put<MO>(acc)
// after them.
template <bool RELU, int TOUT, int RG = 2>
struct EpOut {
  v4 (&o)[TOUT][RG];
  template <int MO>
  __device__ __forceinline__ void pre() {}
  template <int MO>
  __device__ __forceinline__ void put(v4 (&acc)[RG]) {
#pragma unroll
    for (int g = 0; g < RG; ++g) {
      if constexpr (RELU) {
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[g][q] = fmaxf(acc[g][q], 0.f);
      }
      o[MO][g] = acc[g];
    }
  }
};

template <bool INV, int XT, int CT, int TT, int RG = 2>
struct EpAffine {
  v4 (&X)[XT][RG];
  const v4 (&T)[TT][RG];
  float (&ld)[RG];
  template <int MO>
  __device__ __forceinline__ void pre() {}
  template <int MO>
  __device__ __forceinline__ void put(v4 (&s)[RG]) {
#pragma unroll
    for (int g = 0; g < RG; ++g)
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

// M-tile MO of Linear I's biases (the layer's bias block: 16 floats per M-tile
// in slot order), loaded when the tile starts and added after its K-steps, so
// the load's latency hides under them (a bias-initialised accumulator made
// every M-tile's first MFMA wait for memory)
template <class G, int I, int MO>
__device__ __forceinline__ v4 bias_load(const float* __restrict__ bias, int lane) {
  if constexpr (!G::kBias) {
    return v4{0.f, 0.f, 0.f, 0.f};
  } else {
    const float* p = bias + G::bbefore(I) + 16 * MO + 4 * (lane >> 4);
    return v4{p[0], p[1], p[2], p[3]};
  }
}

template <class G, int NETS, int NET, int I, int MO, int TOFF, int P, int TIN, int RG, class EP,
          int... N>
__device__ __forceinline__ void mtile(float (&ring)[P], const float* __restrict__ a,
                                      const float* __restrict__ an,
                                      const float* __restrict__ bias, const v4 (&in)[TIN][RG],
                                      EP& ep, int lane, std::integer_sequence<int, N...>) {
  v4 acc[RG];
#pragma unroll
  for (int g = 0; g < RG; ++g) acc[g] = v4{0.f, 0.f, 0.f, 0.f};
  ep.template pre<MO>();
  const v4 b = bias_load<G, I, MO>(bias, lane);
  (kstep<G, NETS, NET, I, MO, N, TOFF, P>(acc, ring, a, an, in), ...);
  if constexpr (G::kBias) {
#pragma unroll
    for (int g = 0; g < RG; ++g) acc[g] += b;
  }
  ep.template put<MO>(acc);
}

template <class G, int NETS, int NET, int I, int TOFF, int P, int TIN, int RG, class EP, int... M>
__device__ __forceinline__ void lin(float (&ring)[P], const float* __restrict__ a,
                                    const float* __restrict__ an, const float* __restrict__ bias,
                                    const v4 (&in)[TIN][RG], EP& ep, int lane,
                                    std::integer_sequence<int, M...>) {
  (mtile<G, NETS, NET, I, M, TOFF>(ring, a, an, bias, in, ep, lane,
                             std::make_integer_sequence<int, G::ks(I)>{}),
   ...);
}

// One conditioner MLP (stream position NET of the layer) on the state's
// conditioning tiles; its last Linear's tiles go to ep.
template <class G, int NETS, int NET, int P, class EP, int RG>
__device__ __forceinline__ void net(float (&ring)[P], const float* __restrict__ a,
                                    const float* __restrict__ an, const float* __restrict__ bias,
                                    const v4 (&X)[G::XT][RG], EP& ep, int lane) {
  using MS0 = std::make_integer_sequence<int, G::mt(0)>;
  if constexpr (G::NL == 1) {
    lin<G, NETS, NET, 0, 0>(ring, a, an, bias, X, ep, lane, MS0{});
  } else if constexpr (G::NL == 2) {
    v4 h1[G::T1][RG];
    EpOut<true, G::T1, RG> e1{h1};
    lin<G, NETS, NET, 0, 0>(ring, a, an, bias, X, e1, lane, MS0{});
    lin<G, NETS, NET, 1, 0>(ring, a, an, bias, h1, ep, lane,
                         std::make_integer_sequence<int, G::mt(1)>{});
  } else {
    v4 h1[G::T1][RG], h2[G::T2][RG];
    EpOut<true, G::T1, RG> e1{h1};
    EpOut<true, G::T2, RG> e2{h2};
    lin<G, NETS, NET, 0, 0>(ring, a, an, bias, X, e1, lane, MS0{});
    lin<G, NETS, NET, 1, 0>(ring, a, an, bias, h1, e2, lane,
                         std::make_integer_sequence<int, G::mt(1)>{});
    lin<G, NETS, NET, 2, 0>(ring, a, an, bias, h2, ep, lane,
                         std::make_integer_sequence<int, G::mt(2)>{});
  }
}

// state slots -> LDS rows [row][feature]
template <class G, int RG>
__device__ __forceinline__ void put_state(float* st, int S, const v4 (&X)[G::XT][RG], int lane) {
#pragma unroll
  for (int t = 0; t < G::XT; ++t)
#pragma unroll
    for (int g = 0; g < RG; ++g)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int f = feat_of<G>(16 * t + 4 * (lane >> 4) + q);
        if (f >= 0) st[(16 * g + (lane & 15)) * S + f] = X[t][g][q];
      }
}

// state slots <- LDS rows through a gather table (slot of feature f takes
// logical q[f]; q == nullptr: identity)
template <class G, int RG>
__device__ __forceinline__ void get_state(const float* st, int S, const int* qs, v4 (&X)[G::XT][RG],
                                          int lane) {
#pragma unroll
  for (int t = 0; t < G::XT; ++t)
#pragma unroll
    for (int g = 0; g < RG; ++g)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int f = feat_of<G>(16 * t + 4 * (lane >> 4) + q);
        X[t][g][q] = f >= 0 ? st[(16 * g + (lane & 15)) * S + (qs ? qs[f] : f)] : 0.f;
      }
}

template <class G, int RG>
__device__ __forceinline__ void relayout(float* st, int* qs, int S, const int32_t* __restrict__ q,
                                         v4 (&X)[G::XT][RG], int lane) {
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
  // the row mean summed in fp64 and rounded once: the mean torch's fp32
  // reduction approximates (its order is not reproducible here, and a
  // 100-wide flow at N(0, 0.1) turns one ulp of the mean into 1e-2 of the
  // probabilities; tests/test_gpu_parity.py, wide predict at N(0, 0.1))
  double s = 0.0;
  for (int f = f0; f < f1; ++f) s += (double)r[f];
  s += __shfl_xor(s, 32);
  const float mu = (float)(s / D);
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
__global__ __launch_bounds__(64 * kWaves, kRunRG == 2 ? 2 : 1) void k_wide16(
    const float* __restrict__ W, const int32_t* __restrict__ qtab,
    const float* __restrict__ in, float* __restrict__ out, float* __restrict__ ld_out,
    int64_t B, int L, const float* __restrict__ lpri) {
  using G = G16L<D, H1, H2>;
  constexpr bool INV = MODE == 1;
  constexpr int XT = G::XT, CT = G::CT, TT = G::TT;
  constexpr int S = D | 1;  // odd LDS row stride
  constexpr int LSP = G::template lsp<NETS>();
  constexpr int LA = LSP * 64, LF = LA + NETS * G::NB;  // A floats / all floats per layer
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // SGPR: row0, descriptors
  const int64_t row0 = ((int64_t)blockIdx.x * kWaves + wave) * kRunRows;
  // waves synchronise only with themselves (LDS A stream: the whole block
  // takes part in every chunk; a wave past the batch computes zero rows)
  if (!G::kLdsA && row0 >= B) return;
  const int nrows = (int)((B - row0) < kRunRows ? (B - row0) : kRunRows);
  float* st = smem + wave * (kRunRows * S + D);
  int* qs = reinterpret_cast<int*>(st + kRunRows * S);

  // rows -> LDS (coalesced) -> slots
  const float* src = in + row0 * D;
  for (int i = lane; i < kRunRows * D; i += 64) {
    const int r = i / D, f = i - r * D;
    st[r * S + f] = r < nrows ? src[i] : 0.f;
  }
  wsync();
  if constexpr (MODE == 2) {  // x - mean(x) per row (calibrators.py:42)
    for (int rb = 0; rb < kRunRows; rb += 32) row_centre16<D>(st + rb * S, S, lane);
    wsync();
  }
  v4 X[XT][kRunRG];
  get_state<G>(st, S, nullptr, X, lane);
  wsync();

  // the A stream: one ring for the whole launch, P fragments ahead of the MFMAs
  constexpr int P = ring16(LSP, G::kLdsA ? CNF_W16_LDSA_PMAX : CNF_W16_PMAX);
  float ring[P];
  {
    const float* a0 = W + (int64_t)(INV ? L - 1 : 0) * LF + kLaneStride * lane;
    if constexpr (G::kLdsA) {  // chunks 0 and 1 of the first layer, then the ring from LDS
      float* stage = w16_dyn + G::kStateFloats;
#pragma unroll
      for (int k = 0; k < 2 * kAC / 16; ++k)
        __builtin_amdgcn_global_load_lds(const_cast<float*>(a0 + 256 * (4 * k + wave)),
                                         stage + 256 * (4 * k + wave), 16, 0, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
#pragma unroll
      for (int j = 0; j < P; ++j) ring[j] = stage[afrag(j) + 4 * lane];
    } else {
#pragma unroll
      for (int j = 0; j < P; ++j) ring[j] = a0[afrag(j)];
    }
  }
  float ld[kRunRG] = {};
  for (int stp = 0; stp < L; ++stp) {
    const int l = INV ? L - 1 - stp : stp;
    const int ln = stp + 1 < L ? (INV ? l - 1 : l + 1) : l;  // last layer: harmless re-read
    const int32_t* __restrict__ q = qtab + l * D;
    if constexpr (INV) relayout<G>(st, qs, S, q, X, lane);  // flip / rev_perm first
    const float* __restrict__ wl = W + (int64_t)l * LF + kLaneStride * lane;
    const float* __restrict__ wn = W + (int64_t)ln * LF + kLaneStride * lane;
    const float* __restrict__ bl = W + (int64_t)l * LF + LA;  // the layer's bias blocks
    v4 Tv[TT][kRunRG];
    EpOut<false, TT, kRunRG> et{Tv};
    if constexpr (NETS == 2) {  // stream order (prepare): t-net, then s-net
      net<G, 2, 0>(ring, wl, wn, bl, X, et, lane);
      EpAffine<INV, XT, CT, TT, kRunRG> ea{X, Tv, ld};
      net<G, 2, 1>(ring, wl, wn, bl + G::NB, X, ea, lane);
    } else {
      net<G, 1, 0>(ring, wl, wn, bl, X, et, lane);
#pragma unroll
      for (int t = 0; t < TT; ++t)
#pragma unroll
        for (int g = 0; g < kRunRG; ++g) X[CT + t][g] = INV ? X[CT + t][g] - Tv[t][g] : X[CT + t][g] + Tv[t][g];
    }
    pad_steps<G, NETS, P>(ring, wl, wn, std::make_integer_sequence<int, LSP - NETS * G::steps()>{});
    if constexpr (!INV) relayout<G>(st, qs, S, q, X, lane);  // perm then flip
  }
  if constexpr (G::kLdsA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA outlives the block

  // slots -> LDS rows -> coalesced stores
  put_state<G>(st, S, X, lane);
  wsync();
  if constexpr (MODE == 2) {
    for (int rb = 0; rb < kRunRows; rb += 32) row_predict16<D>(st + rb * S, S, lane, lpri);
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
  for (int g = 0; g < kRunRG; ++g) {
    ld[g] += __shfl_xor(ld[g], 16);
    ld[g] += __shfl_xor(ld[g], 32);
  }
  if (ld_out && lane < 16) {
#pragma unroll
    for (int g = 0; g < kRunRG; ++g)
      if (16 * g + lane < nrows) ld_out[row0 + 16 * g + lane] = ld[g];
  }
}

// ---------------------------------------------------------------------------
// Training (cnf_vjp / cnf_loss_vjp of these shapes): the forward sweep as
// above plus a per-row tape, then one reverse-sweep launch per layer whose
// transposed products run on the same register tiles.  Replaces autograd of
// flows/flows.py:101-112 and flows/utils.py:26-31 for the stacks in the table.
// ---------------------------------------------------------------------------

// Reverse-mode chain of one conditioner, last Linear first: step i is the
// transposed product of forward Linear f = NL-1-i (input: the gradient of f's
// output, nout_f units; output: the gradient of f's input, nin_f units).  No
// biases: accumulators start at 0.
template <int D, int H1, int H2>
struct G16T {
  using F = G16<D, H1, H2>;
  static constexpr bool kBias = false;
  static constexpr bool kLdsA = false;
  static constexpr int DT = F::DT, DC = F::DC, NL = F::NL, CT = F::CT, TT = F::TT, XT = F::XT;
  static constexpr int nin(int i) { return F::nout(NL - 1 - i); }
  static constexpr int nout(int i) { return F::nin(NL - 1 - i); }
  static constexpr int ks(int i) { return cdiv(nin(i), 4); }
  static constexpr int mt(int i) { return cdiv(nout(i), 16); }
  static constexpr int sbefore(int i) { return i == 0 ? 0 : sbefore(i - 1) + mt(i - 1) * ks(i - 1); }
  static constexpr int steps() { return sbefore(NL); }
  static constexpr int bbefore(int) { return 0; }
  static constexpr int NA = steps() * 64;
  // The reverse sweep's stream per layer is padded to a multiple of 16 steps
  // (a few fragments no MFMA uses): the A ring, which must divide the layer's
  // steps, can then be 16 deep instead of 12, and every tape / G access gets 16
  // K-steps to complete before a ring wait covers it (vmcnt counts in order).
  template <int NETS>
  static constexpr int lsp() { return pad_ls(NETS * steps(), CNF_W16_BWD_P16); }
};


// Per-row tape of one layer, every part in slot order (16-slot tiles), so the
// reverse sweep reads back exactly the register tiles the forward held:
//   XC  conditioning half, 1 at unit DC (the bias column of dW)  16 cdiv(DC+1, 16)
//   XT  transformed half before the update                       16 TT
//   S   the s-net's output (NETS == 2)                           16 TT
//   H   per net n, hidden k = 1..NL-1: relu(h_k), 1 at unit H_k  16 cdiv(H_k+1, 16)
// and the reverse sweep's per-row conditioner gradients (the dW operands):
//   per net n: G_last (of its output, 16 TT), then per hidden k the gradient of
//   h_k's pre-activation (16 cdiv(H_k, 16)).
// Nets in natural order: 0 the s-net, 1 the t-net (NETS == 1: the t-net).
template <int D, int H1, int H2, int NETS>
struct Tape16 {
  using F = G16<D, H1, H2>;
  static constexpr int CW = 16 * cdiv(F::DC + 1, 16);
  static constexpr int TS = 16 * F::TT;
  static constexpr int HW(int k) { return 16 * cdiv(F::hid(k) + 1, 16); }
  static constexpr int XC = 0, XTo = CW, So = CW + TS;
  static constexpr int H0 = So + (NETS == 2 ? TS : 0);
  static constexpr int netH = (F::NL > 1 ? HW(1) : 0) + (F::NL > 2 ? HW(2) : 0);
  static constexpr int H(int n, int k) { return H0 + n * netH + (k == 2 ? HW(1) : 0); }
  static constexpr int RW = 16 * cdiv(H0 + NETS * netH, 16);
  static constexpr int GP(int k) { return 16 * cdiv(F::hid(k), 16); }
  static constexpr int netG = TS + (F::NL > 1 ? GP(1) : 0) + (F::NL > 2 ? GP(2) : 0);
  static constexpr int Glast(int n) { return n * netG; }
  static constexpr int Gpre(int n, int k) { return n * netG + TS + (k == 2 ? GP(1) : 0); }
  static constexpr int GW = NETS * netG;
};

typedef int v4i __attribute__((ext_vector_type(4)));

// A/B knobs: which tape traffic runs (never shipped changed) -- bit 0 the
// XC / XT / S stores, 1 the hidden stores, 2 the reverse sweep's G stores --
// and the stores' cache-policy bits (nt measured 0.45 ms faster per forward
// sweep and 0.36 ms per reverse sweep at cfg4 than default-policy stores)
#ifndef CNF_W16_TAPE
#define CNF_W16_TAPE 15
#endif
#ifndef CNF_W16_STORE_AUX
#define CNF_W16_STORE_AUX 2  // nt: streaming stores (tape reuse is a whole sweep away)
#endif

// One wave's block of a wave-tiled [B][W] array (the tape and G layouts):
// rows in blocks of 32, a block's 32 x W floats as [W / 16 tiles][2 row
// groups][16 rows][16 slots], so row r = 32 w + 16 g + i, column c sits at
//   w * 32 W + (c >> 4) * 512 + g * 256 + i * 16 + (c & 15)
// and one tile store of a row group is one contiguous KiB (row-major [B][W]
// rows took 64-B pieces of 16 rows per store: 0.68 ms more per cfg4 forward
// sweep).  Lane (i, k) of row group g addresses row 16 g + i, slots 4k..4k+3.
// Arrays are allocated in whole blocks: a ragged wave's rows past the batch
// read and write the padding.
struct Rows16 {
  __amdgpu_buffer_rsrc_t rs;
  int voff[2];
  // live = false: a wave wholly past the batch (it still runs the block's
  // stream for the LDS A-stream barriers): every access falls outside the
  // descriptor (stores dropped, loads read 0)
  __device__ __forceinline__ Rows16(const float* block, int W, int lane, bool live = true) {
    rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(block), 0, live ? kRows * W * 4 : 0,
                                           0x00020000);
#pragma unroll
    for (int g = 0; g < 2; ++g) voff[g] = (g * 256 + (lane & 15) * 16 + 4 * (lane >> 4)) * 4;
  }
  // off: the tile's first slot (floats into the row, a multiple of 16)
  __device__ __forceinline__ void store(const v4& v, int g, int off) const {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v), rs, voff[g], off * 128,
                                           CNF_W16_STORE_AUX);
  }
  __device__ __forceinline__ v4 load(int g, int off) const {
    return __builtin_bit_cast(v4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff[g], off * 128, 0));
  }
};

// slot ONE of a tile set to 1 in lane group (ONE >> 2) & 3 (the ones column)
template <int ONE, int MO>
__device__ __forceinline__ v4 with_one(v4 v, int lane) {
  if constexpr ((ONE >> 4) == MO) {
    if ((lane >> 4) == ((ONE >> 2) & 3)) v[ONE & 3] = 1.f;
  }
  return v;
}

// Tape traffic and the vector-memory counter.  A wave waits for its A-ring
// loads with vmcnt, which counts loads and stores alike and in issue order:
// every store or tape load must complete within the P K-steps that separate
// a ring load from its use, or it stalls the MFMA stream (measured: per-tile
// stores and relu' loads cost the reverse sweep 156 us per cfg4 layer, the
// forward's hidden stores 97 us).  So the sweeps issue tape stores in bursts,
// one per Linear (the tiles are live anyway: the next Linear's input), and
// the reverse sweep takes relu' from BITS written by the forward -- one bit
// per activation, every hidden layer of a layer in 8 words per lane, loaded
// once when the launch starts -- instead of loading the activations per tile.

// relu' bits of hidden layer word pair WI (4 words per net and lane): bit
// 8 (MO & 3) + 4 g + q of word WI + (MO >> 2) is (h > 0) for register q, row
// group g of M-tile MO (hidden widths up to 128)
template <int WI, int MO>
__device__ __forceinline__ void put_bits(uint32_t (&mb)[4], const v4 (&h)[2]) {
  static_assert(MO < 8, "relu' bits cover 8 tiles");
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (h[g][q] > 0.f) mb[WI + (MO >> 2)] |= 1u << (8 * (MO & 3) + 4 * g + q);
}
template <int WI, int MO>
__device__ __forceinline__ bool get_bit(const uint32_t (&mb)[8], int g, int q) {
  return (mb[WI + (MO >> 2)] >> (8 * (MO & 3) + 4 * g + q)) & 1u;
}

// hidden Linear of the forward sweep: ReLU, keep the tile, record relu'
template <int TOUT, int WI>
struct EpTape {
  v4 (&o)[TOUT][2];
  uint32_t (&mb)[4];
  template <int MO>
  __device__ __forceinline__ void pre() {}
  template <int MO>
  __device__ __forceinline__ void put(v4 (&acc)[2]) {
#pragma unroll
    for (int g = 0; g < 2; ++g) {
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[g][q] = fmaxf(acc[g][q], 0.f);
      o[MO][g] = acc[g];
    }
    put_bits<WI, MO>(mb, acc);
  }
};

// one burst of T tiles into part OFF (slot ONE of the part set to 1)
template <int OFF, int T, int ONE>
__device__ __forceinline__ void tape_tiles(const Rows16& tp, const v4 (&h)[T][2], int lane) {
  if (!(CNF_W16_TAPE & 2)) return;
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      v4 v = h[t][g];
      if ((ONE >> 4) == t && (lane >> 4) == ((ONE >> 2) & 3)) v[ONE & 3] = 1.f;
      tp.store(v, g, OFF + 16 * t);
    }
}

// a part's extra tile holding only the ones column (width a multiple of 16)
template <int OFF, int T, int ONE>
__device__ __forceinline__ void tape_ones_tile(const Rows16& tp, int lane) {
  if constexpr ((ONE >> 4) == T) {
#pragma unroll
    for (int g = 0; g < 2; ++g) tp.store(with_one<ONE, T>(v4{0.f, 0.f, 0.f, 0.f}, lane), g, OFF + 16 * T);
  }
}

// the s-net's last Linear: tape s, then the affine update (as EpAffine)
template <int XT, int CT, int TT, int OFF>
struct EpAffineTape {
  v4 (&X)[XT][2];
  const v4 (&T)[TT][2];
  float (&ld)[2];
  const Rows16& tp;
  template <int MO>
  __device__ __forceinline__ void pre() {}
  template <int MO>
  __device__ __forceinline__ void put(v4 (&s)[2]) {
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      if (CNF_W16_TAPE & 1) tp.store(s[g], g, OFF + 16 * MO);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float sv = s[g][q];
        const float e = __builtin_amdgcn_exp2f(sv * 1.4426950408889634f);
        X[CT + MO][g][q] = fmaf(X[CT + MO][g][q], e, T[MO][g][q]);
        ld[g] += sv;
      }
    }
  }
};

// One conditioner of the forward sweep (stream position POS, tape net N)
// (relu' bits of hidden k: words 2 (k - 1), +1 of the net's four, stored to
// bits[4 N ..] of the wave's lane record when the net is done)
template <class G, class TP, int NETS, int POS, int N, int P, class EP>
__device__ __forceinline__ void net_tape(float (&ring)[P], const float* __restrict__ a,
                                         const float* __restrict__ an,
                                         const float* __restrict__ bias,
                                         const v4 (&X)[G::XT][2], EP& ep, const Rows16& tp,
                                         uint32_t* __restrict__ bits, int lane) {
  using MS0 = std::make_integer_sequence<int, G::mt(0)>;
  if constexpr (G::NL == 1) {
    lin<G, NETS, POS, 0, 0>(ring, a, an, bias, X, ep, lane, MS0{});
  } else {
    uint32_t mb[4] = {0u, 0u, 0u, 0u};
    constexpr int O1 = qslot(G::hid(1));
    v4 h1[G::T1][2];
    EpTape<G::T1, 0> e1{h1, mb};
    lin<G, NETS, POS, 0, 0>(ring, a, an, bias, X, e1, lane, MS0{});
    tape_tiles<TP::H(N, 1), G::T1, O1>(tp, h1, lane);
    tape_ones_tile<TP::H(N, 1), G::T1, O1>(tp, lane);
    if constexpr (G::NL == 2) {
      lin<G, NETS, POS, 1, 0>(ring, a, an, bias, h1, ep, lane,
                              std::make_integer_sequence<int, G::mt(1)>{});
    } else {
      constexpr int O2 = qslot(G::hid(2));
      v4 h2[G::T2][2];
      EpTape<G::T2, 2> e2{h2, mb};
      lin<G, NETS, POS, 1, 0>(ring, a, an, bias, h1, e2, lane,
                              std::make_integer_sequence<int, G::mt(1)>{});
      tape_tiles<TP::H(N, 2), G::T2, O2>(tp, h2, lane);
      tape_ones_tile<TP::H(N, 2), G::T2, O2>(tp, lane);
      lin<G, NETS, POS, 2, 0>(ring, a, an, bias, h2, ep, lane,
                              std::make_integer_sequence<int, G::mt(2)>{});
    }
    if (bits) *reinterpret_cast<v4i*>(bits + 4 * N) = v4i{(int)mb[0], (int)mb[1], (int)mb[2], (int)mb[3]};
  }
}

// The loss seed of a wave's 32 rows (z_L in LDS, natural order; the
// calibrator NLL or CE of calibrators.py:287-291 / run_experiment3D.py:102-107,
// as k_wseed in cnf_wvjp.hip): lane (r, h) = (lane & 31, lane >> 5) takes
// half of row r's features.  Writes the gradient of z_L into the LDS rows,
// gld per row, and the wave's (loss, ce, ld) sums to part[0..2] (fixed
// order: deterministic).
struct SeedArgs {
  const int64_t* y;
  float* G;     // [B][D] gradient of z_L
  float* gld;   // [B]
  float* part;  // [waves][4]
  float det, grad_scale;
  int kind;     // CNF_LOSS_*, or < 0: no seed (the final output goes to zst)
};
template <int D>
__device__ __forceinline__ void row_seed(float* st, int S, int lane, int64_t row0, int nrows,
                                         float ldr, const SeedArgs& a) {
  constexpr int HF = (D + 1) / 2;
  const int row = lane & 31, f0 = (lane >> 5) * HF, f1 = f0 + HF < D ? f0 + HF : D;
  const bool valid = row < nrows;
  float* r = st + row * S;
  float m = -__builtin_inff();
  for (int f = f0; f < f1; ++f) m = fmaxf(m, r[f]);
  m = fmaxf(m, __shfl_xor(m, 32));
  float se = 0.f;
  for (int f = f0; f < f1; ++f) se += expf(r[f] - m);
  se += __shfl_xor(se, 32);
  const float lse = m + logf(se);
  const int64_t yy = valid ? a.y[row0 + row] : 0;
  const bool ok = yy >= 0 && yy < D;
  const int yi = ok ? (int)yy : 0;
  const float lpy = r[yi] - lse;
  float coef, ce, loss, gl;
  if (a.kind == CNF_LOSS_CAL) {  // -(log(softmax(z)[y] + 1e-7) + ld)
    const float py = expf(lpy);
    ce = -logf(py + 1e-7f);
    loss = ce - ldr;
    coef = py / (py + 1e-7f);
    gl = -a.grad_scale;
  } else {  // CE(z, y) - det * ld
    ce = -lpy;
    loss = ce - a.det * ldr;
    coef = 1.f;
    gl = -a.det * a.grad_scale;
  }
  if (!ok) ce = loss = coef = __builtin_nanf("");
  wsync();  // every lane has read r[yi] before the row is overwritten
  const float sc = a.grad_scale * coef;
  for (int f = f0; f < f1; ++f) r[f] = sc * (expf(r[f] - lse) - (f == yi ? 1.f : 0.f));
  if (valid && lane < 32) a.gld[row0 + row] = gl;
  float s0 = valid && lane < 32 ? loss : 0.f, s1 = valid && lane < 32 ? ce : 0.f,
        s2 = valid && lane < 32 ? ldr : 0.f;
#pragma unroll
  for (int o = 16; o >= 1; o >>= 1) {
    s0 += __shfl_xor(s0, o);
    s1 += __shfl_xor(s1, o);
    s2 += __shfl_xor(s2, o);
  }
  if (lane == 0) {
    float* p = a.part + (row0 / kRows) * 4;
    p[0] = s0;
    p[1] = s1;
    p[2] = s2;
    p[3] = 0.f;
  }
}

// Forward sweep of training: k_wide16's forward with the tape of every layer
// written on the way, then either the loss seed (sa.kind >= 0: the gradient of
// z_L, gld and the loss sums, as k_wseed) or the final output in the stash
// layout k_wseed reads (column Cp + f for f < DT, f - DT otherwise; row stride
// Dp) and each row's log-det.
template <int D, int H1, int H2, int NETS>
__global__ __launch_bounds__(64 * kWaves, 2) void k_wtrain16_fwd(
    const float* __restrict__ W, const int32_t* __restrict__ qtab, const float* __restrict__ in,
    float* __restrict__ zst, float* __restrict__ ld_out, float* __restrict__ tape,
    uint32_t* __restrict__ tbits, int64_t B, int L, int Cp, int Dp, SeedArgs sa) {
  using G = std::conditional_t<CNF_W16_TRAIN_LDSA != 0 && kRunRows == kRows, G16L<D, H1, H2>,
                               G16<D, H1, H2>>;
  using TP = Tape16<D, H1, H2, NETS>;
  constexpr int XT = G::XT, CT = G::CT, TT = G::TT;
  constexpr int S = D | 1;
  constexpr int LSP = G::template lsp<NETS>();
  constexpr int LA = LSP * 64, LF = LA + NETS * G::NB;
  constexpr int OC = qslot(G::DC);
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // SGPR: row0, descriptors
  const int64_t row0 = ((int64_t)blockIdx.x * kWaves + wave) * kRows;
  // (LDS A stream: the whole block meets every chunk barrier; a wave past the
  // batch runs the stream on zero rows with its tape descriptors empty)
  if (!G::kLdsA && row0 >= B) return;
  const bool live = row0 < B;
  const int nrows = !live ? 0 : (int)((B - row0) < kRows ? (B - row0) : kRows);
  const int64_t nwb = (B + kRows - 1) / kRows;
  float* st = smem + wave * (kRows * S + D);
  int* qs = reinterpret_cast<int*>(st + kRows * S);

  const float* src = in + row0 * D;
  for (int i = lane; i < kRows * D; i += 64) {
    const int r = i / D, f = i - r * D;
    st[r * S + f] = r < nrows ? src[i] : 0.f;
  }
  wsync();
  v4 X[XT][2];
  get_state<G>(st, S, nullptr, X, lane);
  wsync();

  constexpr int P = ring16(LSP, G::kLdsA ? CNF_W16_LDSA_PMAX : CNF_W16_PMAX);
  float ring[P];
  if constexpr (G::kLdsA) {  // chunks 0 and 1 of the first layer, then the ring from LDS
    float* stage = w16_dyn + G::kStateFloats;
#pragma unroll
    for (int k = 0; k < 2 * kAC / 16; ++k)
      __builtin_amdgcn_global_load_lds(const_cast<float*>(W + kLaneStride * lane + 256 * (4 * k + wave)),
                                       stage + 256 * (4 * k + wave), 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (int j = 0; j < P; ++j) ring[j] = stage[afrag(j) + 4 * lane];
  } else {
#pragma unroll
    for (int j = 0; j < P; ++j) ring[j] = W[kLaneStride * lane + afrag(j)];
  }
  float ld[2] = {0.f, 0.f};
  for (int l = 0; l < L; ++l) {
    const int ln = l + 1 < L ? l + 1 : l;
    const float* __restrict__ wl = W + (int64_t)l * LF + kLaneStride * lane;
    const float* __restrict__ wn = W + (int64_t)ln * LF + kLaneStride * lane;
    const float* __restrict__ bl = W + (int64_t)l * LF + LA;
    const Rows16 tp(tape + ((int64_t)l * nwb * kRows + (live ? row0 : 0)) * TP::RW, TP::RW, lane,
                    live);
#pragma unroll
    for (int g = 0; g < 2; ++g) {
#pragma unroll
      for (int t = 0; t < CT; ++t) {
        v4 v = X[t][g];
        if ((OC >> 4) == t && (lane >> 4) == ((OC >> 2) & 3)) v[OC & 3] = 1.f;
        if (CNF_W16_TAPE & 1) tp.store(v, g, TP::XC + 16 * t);
      }
#pragma unroll
      for (int t = 0; t < TT; ++t)
        if (CNF_W16_TAPE & 1) tp.store(X[CT + t][g], g, TP::XTo + 16 * t);
    }
    tape_ones_tile<TP::XC, CT, OC>(tp, lane);
    v4 Tv[TT][2];
    EpOut<false, TT> et{Tv};
    // this wave's relu' bits: 8 words per lane (4 per net)
    // (a wave past the batch writes its bits into block 0's record of this
    // layer ... never: net_tape stores them only when `bp` is non-null)
    uint32_t* bp = live ? tbits + ((int64_t)l * nwb + row0 / kRows) * 512 + lane * 8 : nullptr;
    if constexpr (NETS == 2) {  // forward stream: t-net (tape net 1), then s-net (net 0)
      net_tape<G, TP, 2, 0, 1>(ring, wl, wn, bl, X, et, tp, bp, lane);
      EpAffineTape<XT, CT, TT, TP::So> ea{X, Tv, ld, tp};
      net_tape<G, TP, 2, 1, 0>(ring, wl, wn, bl + G::NB, X, ea, tp, bp, lane);
    } else {
      net_tape<G, TP, 1, 0, 0>(ring, wl, wn, bl, X, et, tp, bp, lane);
#pragma unroll
      for (int t = 0; t < TT; ++t)
#pragma unroll
        for (int g = 0; g < 2; ++g) X[CT + t][g] = X[CT + t][g] + Tv[t][g];
    }
    pad_steps<G, NETS, P>(ring, wl, wn, std::make_integer_sequence<int, LSP - NETS * G::steps()>{});
    relayout<G>(st, qs, S, qtab + l * D, X, lane);
  }
  if constexpr (G::kLdsA) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA outlives the block
    if (!live) return;
  }

  put_state<G>(st, S, X, lane);
  wsync();
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    ld[g] += __shfl_xor(ld[g], 16);
    ld[g] += __shfl_xor(ld[g], 32);
  }
  if (sa.kind >= 0) {
    // lane l holds row (l & 15)'s log-det in ld[0] and row 16 + (l & 15)'s in ld[1]
    row_seed<D>(st, S, lane, row0, nrows, (lane & 16) ? ld[1] : ld[0], sa);
    wsync();
    float* dst = sa.G + row0 * D;
    for (int i = lane; i < nrows * D; i += 64) {
      const int r = i / D, f = i - r * D;
      dst[i] = st[r * S + f];
    }
    return;
  }
  for (int i = lane; i < nrows * D; i += 64) {
    const int r = i / D, f = i - r * D;
    zst[(row0 + r) * Dp + (f < G::DT ? Cp + f : f - G::DT)] = st[r * S + f];
  }
  if (lane < 16) {
#pragma unroll
    for (int g = 0; g < 2; ++g)
      if (16 * g + lane < nrows) ld_out[row0 + 16 * g + lane] = ld[g];
  }
}

// reverse sweep, hidden step: relu'(h) from the forward's bits (torch's
// threshold backward: h <= 0 -> 0), keep the tile (stored as a dW operand in
// one burst after the Linear)
template <int TOUT, int WI>
struct EpMaskTape {
  v4 (&o)[TOUT][2];
  const uint32_t (&mb)[8];
  template <int MO>
  __device__ __forceinline__ void pre() {}
  template <int MO>
  __device__ __forceinline__ void put(v4 (&acc)[2]) {
#pragma unroll
    for (int g = 0; g < 2; ++g) {
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[g][q] = get_bit<WI, MO>(mb, g, q) ? acc[g][q] : 0.f;
      o[MO][g] = acc[g];
    }
  }
};

template <int OFF, int T>
__device__ __forceinline__ void g_tiles(const Rows16& gb, const v4 (&h)[T][2]) {
  if (!(CNF_W16_TAPE & 4)) return;
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int g = 0; g < 2; ++g) gb.store(h[t][g], g, OFF + 16 * t);
}

// reverse sweep, first Linear: the conditioners' share of the gradient of the
// conditioning half, added to the state's tiles
template <int XT>
struct EpAddC {
  v4 (&X)[XT][2];
  template <int MO>
  __device__ __forceinline__ void pre() {}
  template <int MO>
  __device__ __forceinline__ void put(v4 (&acc)[2]) {
#pragma unroll
    for (int g = 0; g < 2; ++g) X[MO][g] = X[MO][g] + acc[g];
  }
};

// Back through one conditioner (net N, reverse-stream position N) from the
// gradient of its output (tiles TOFF.. of `in`) into the state's C tiles.
template <class GT, class TP, int NETS, int N, int TOFF, int P, int TIN, int XT>
__device__ __forceinline__ void net_back(float (&ring)[P], const float* __restrict__ a,
                                         const float* __restrict__ an,
                                         const v4 (&in)[TIN][2], v4 (&X)[XT][2],
                                         const uint32_t (&mb)[8], const Rows16& gb, int lane) {
  EpAddC<XT> ec{X};
  using MS0 = std::make_integer_sequence<int, GT::mt(0)>;
  if constexpr (GT::NL == 1) {
    lin<GT, NETS, N, 0, TOFF>(ring, a, an, nullptr, in, ec, lane, MS0{});
  } else if constexpr (GT::NL == 2) {
    v4 g1[GT::mt(0)][2];
    EpMaskTape<GT::mt(0), 4 * N> e0{g1, mb};
    lin<GT, NETS, N, 0, TOFF>(ring, a, an, nullptr, in, e0, lane, MS0{});
    g_tiles<TP::Gpre(N, 1), GT::mt(0)>(gb, g1);
    lin<GT, NETS, N, 1, 0>(ring, a, an, nullptr, g1, ec, lane,
                           std::make_integer_sequence<int, GT::mt(1)>{});
  } else {
    v4 g2[GT::mt(0)][2];
    EpMaskTape<GT::mt(0), 4 * N + 2> e0{g2, mb};
    lin<GT, NETS, N, 0, TOFF>(ring, a, an, nullptr, in, e0, lane, MS0{});
    g_tiles<TP::Gpre(N, 2), GT::mt(0)>(gb, g2);
    v4 g1[GT::mt(1)][2];
    EpMaskTape<GT::mt(1), 4 * N> e1{g1, mb};
    lin<GT, NETS, N, 1, 0>(ring, a, an, nullptr, g2, e1, lane,
                           std::make_integer_sequence<int, GT::mt(1)>{});
    g_tiles<TP::Gpre(N, 1), GT::mt(1)>(gb, g1);
    lin<GT, NETS, N, 2, 0>(ring, a, an, nullptr, g1, ec, lane,
                           std::make_integer_sequence<int, GT::mt(2)>{});
  }
}

// The reverse sweep, every layer in one launch (last first), 32 rows per wave;
// the gradient state stays in registers from layer to layer and the A ring
// runs on from one layer's transposed stream into the next.  Per layer l:
//   g_out (+ the caller's gradient of z_l when l < L-1) is gathered back
//   through the flip / permutation (iq = fq^-1, one LDS pass);
//   with e = e^s:  G_s = g_T x_T e + gld,  G_t = g_T,  g_in_T = g_T e,
//   g_in_C = g_C + the conditioners' share (their transposed chains, relu'
//   from the forward's bits).
// Every Linear's output gradient goes to layer l's G rows (the dW operands).
// gz: the seed (gradient of z_{L-1}, natural order); dx (optional): the
// gradient of the flow's input.
template <int D, int H1, int H2, int NETS>
__global__ __launch_bounds__(64 * kWaves, 2) void k_wtrain16_bwd(
    const float* __restrict__ WT, const int32_t* __restrict__ iqtab, const float* __restrict__ gz,
    const float* __restrict__ gz_all, float* __restrict__ dx, const float* __restrict__ gld,
    const float* __restrict__ tape, const uint32_t* __restrict__ tbits, float* __restrict__ gbuf,
    int64_t B, int L) {
  using G = G16<D, H1, H2>;
  using GT = G16T<D, H1, H2>;
  using TP = Tape16<D, H1, H2, NETS>;
  constexpr int XT = G::XT, CT = G::CT, TT = G::TT;
  constexpr int S = D | 1;
  constexpr int LSP = GT::template lsp<NETS>();
  constexpr int LT = LSP * 64;  // transposed-stream floats per layer (pads included)
  constexpr float kL2E = 1.4426950408889634f;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // SGPR: row0, descriptors
  const int64_t row0 = ((int64_t)blockIdx.x * kWaves + wave) * kRows;
  if (row0 >= B) return;
  const int nrows = (int)((B - row0) < kRows ? (B - row0) : kRows);
  const int64_t nwb = (B + kRows - 1) / kRows;
  float* st = smem + wave * (kRows * S + D);
  int* qs = reinterpret_cast<int*>(st + kRows * S);

  const float* src = gz + row0 * D;
  for (int i = lane; i < kRows * D; i += 64) {
    const int r = i / D, f = i - r * D;
    st[r * S + f] = r < nrows ? src[i] : 0.f;
  }
  constexpr int P = ring16(LSP, CNF_W16_PMAX);
  float ring[P];
  {
    const float* a0 = WT + (int64_t)(L - 1) * LT + kLaneStride * lane;
#pragma unroll
    for (int j = 0; j < P; ++j) ring[j] = a0[afrag(j)];
  }
  float gl[2];
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int r = 16 * g + (lane & 15);
    gl[g] = r < nrows ? gld[row0 + r] : 0.f;
  }
  v4 X[XT][2];
  for (int l = L - 1; l >= 0; --l) {
    // this layer's relu' bits (issued first, used late)
    uint32_t mb[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
    if constexpr (G::NL > 1) {
      const uint32_t* bp = tbits + ((int64_t)l * nwb + row0 / kRows) * 512 + lane * 8;
      const v4i b0 = *reinterpret_cast<const v4i*>(bp);
      mb[0] = b0[0], mb[1] = b0[1], mb[2] = b0[2], mb[3] = b0[3];
      if constexpr (NETS == 2) {
        const v4i b1 = *reinterpret_cast<const v4i*>(bp + 4);
        mb[4] = b1[0], mb[5] = b1[1], mb[6] = b1[2], mb[7] = b1[3];
      }
    }
    const Rows16 tp(tape + ((int64_t)l * nwb * kRows + row0) * TP::RW, TP::RW, lane);
    const Rows16 gb(gbuf + ((int64_t)l * nwb * kRows + row0) * TP::GW, TP::GW, lane);
    v4 xv[TT][2], sv[TT][2];
#pragma unroll
    for (int t = 0; t < TT; ++t)
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        xv[t][g] = tp.load(g, TP::XTo + 16 * t);
        if constexpr (NETS == 2) sv[t][g] = tp.load(g, TP::So + 16 * t);
      }
    // g_out of layer l in LDS (natural order): the caller's gradient of z_l
    // joins it, then the gather through iq
    for (int j = lane; j < D; j += 64) qs[j] = iqtab[l * D + j];
    if (gz_all && l < L - 1) {
      const float* gp = gz_all + ((int64_t)l * B + row0) * D;
      for (int i = lane; i < nrows * D; i += 64) {
        const int r = i / D, f = i - r * D;
        st[r * S + f] += gp[i];
      }
    }
    wsync();
    get_state<G>(st, S, qs, X, lane);
    wsync();
    const float* __restrict__ wa = WT + (int64_t)l * LT + kLaneStride * lane;
    const float* __restrict__ wn = WT + (int64_t)(l > 0 ? l - 1 : l) * LT + kLaneStride * lane;
    if constexpr (NETS == 2) {
      v4 Gs[TT][2];
#pragma unroll
      for (int t = 0; t < TT; ++t)
#pragma unroll
        for (int g = 0; g < 2; ++g) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float e = __builtin_amdgcn_exp2f(sv[t][g][q] * kL2E);
            const bool real = 16 * t + 4 * q + (lane >> 4) < G::DT;
            Gs[t][g][q] = real ? __fadd_rn(__fmul_rn(__fmul_rn(X[CT + t][g][q], xv[t][g][q]), e), gl[g])
                               : 0.f;
          }
          gb.store(Gs[t][g], g, TP::Glast(0) + 16 * t);
          gb.store(X[CT + t][g], g, TP::Glast(1) + 16 * t);
        }
      net_back<GT, TP, 2, 0, 0>(ring, wa, wn, Gs, X, mb, gb, lane);   // s-net
      net_back<GT, TP, 2, 1, CT>(ring, wa, wn, X, X, mb, gb, lane);   // t-net: G_t = g_T
      // g_in_T = g_T e (s reloaded: the tape part is read-only here)
#pragma unroll
      for (int t = 0; t < TT; ++t)
#pragma unroll
        for (int g = 0; g < 2; ++g) sv[t][g] = tp.load(g, TP::So + 16 * t);
#pragma unroll
      for (int t = 0; t < TT; ++t)
#pragma unroll
        for (int g = 0; g < 2; ++g)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            X[CT + t][g][q] = __fmul_rn(X[CT + t][g][q], __builtin_amdgcn_exp2f(sv[t][g][q] * kL2E));
    } else {
#pragma unroll
      for (int t = 0; t < TT; ++t)
#pragma unroll
        for (int g = 0; g < 2; ++g) gb.store(X[CT + t][g], g, TP::Glast(0) + 16 * t);
      net_back<GT, TP, 1, 0, CT>(ring, wa, wn, X, X, mb, gb, lane);
    }
    pad_steps<GT, NETS, P>(ring, wa, wn, std::make_integer_sequence<int, LSP - NETS * GT::steps()>{});
    put_state<G>(st, S, X, lane);  // g_in: the gradient of z_{l-1} (natural order)
    wsync();
  }
  if (dx) {
    float* dst = dx + row0 * D;
    for (int i = lane; i < nrows * D; i += 64) {
      const int r = i / D, f = i - r * D;
      dst[i] = st[r * S + f];
    }
  }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
using WFn = void (*)(const float*, const int32_t*, const float*, float*, float*, int64_t, int,
                    const float*);
using TFwdFn = void (*)(const float*, const int32_t*, const float*, float*, float*, float*,
                        uint32_t*, int64_t, int, int, int, SeedArgs);
using TBwdFn = void (*)(const float*, const int32_t*, const float*, const float*, float*,
                        const float*, const float*, const uint32_t*, float*, int64_t, int);

// One Linear's A / bias recipe for the prepare kernel.
struct WSeg16 {
  const float* W;
  const float* b;
  int64_t abase;          // float offset of the layer's stream (step 0)
  int64_t adst, bdst;     // float offsets of its A fragments and bias block (-1: none)
  int nm, nk;             // M-tiles, K-steps
  int first;              // the Linear reads the conditioning half (weight columns DT..D-1)
  int trans;              // the transposed product (reverse sweep): out = the Linear's input
  int nin, nout;          // real input / output units of the product
  int nin_full;           // the reference weight is [nout][nin_full] (forward sense)
  int DT;
};
struct WPrep16 {
  WSeg16 seg[12];  // 2 nets x up to 3 Linears, forward and transposed
  int nseg;
};

// A fragment (M-tile mo, K-step n), lane l: product output unit o = qslot(16 mo
// + (l & 15)), input unit u = 4 n + (l >> 4): W[o][u] (forward) or W[u][o]
// (transposed); bias block: slot order, zero at padding slots.
__global__ void k_prepare_wide16(WPrep16 a, float* __restrict__ wreg) {
  const WSeg16& g = a.seg[blockIdx.x];
  const int64_t n = (int64_t)g.nm * g.nk * 64;
  const int c0 = g.first ? g.DT : 0;
  for (int64_t e = threadIdx.x + (int64_t)blockIdx.y * blockDim.x; e < n;
       e += (int64_t)blockDim.x * gridDim.y) {
    const int lane = (int)(e & 63), ks = (int)((e >> 6) % g.nk), mo = (int)((e >> 6) / g.nk);
    const int o = qslot(16 * mo + (lane & 15)), u = 4 * ks + (lane >> 4);
    float v = 0.f;
    if (o < g.nout && u < g.nin)
      v = g.trans ? g.W[(int64_t)u * g.nin_full + c0 + o] : g.W[(int64_t)o * g.nin_full + c0 + u];
    const int64_t x = g.adst - g.abase + e;  // fragment-major offset in the stream
    wreg[g.abase + afrag((int)(x >> 6)) + kLaneStride * (x & 63)] = v;
  }
  if (g.bdst < 0 || blockIdx.y != 0) return;
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
  TFwdFn tfwd[2];  // [nets - 1] training sweeps
  TBwdFn tbwd[2];
  int nat;         // transposed A floats per net and layer
  int ksT[3], mtT[3], abeforeT[3];  // per reverse step i (forward Linear NL-1-i)
  WTrain16Layout lay[2];  // [nets - 1]
};

#define CNF_G16(D, H1, H2) G16<D, H1, H2>
#define CNF_G16T(D, H1, H2) G16T<D, H1, H2>

template <int D, int H1, int H2, int NETS>
constexpr WTrain16Layout train_layout() {
  using TP = Tape16<D, H1, H2, NETS>;
  using F = G16<D, H1, H2>;
  WTrain16Layout y{};
  y.RW = TP::RW;
  y.GW = TP::GW;
  y.xc = TP::XC;
  y.cw = TP::CW;
  y.xt = TP::XTo;
  y.s = NETS == 2 ? TP::So : -1;
  y.ts = TP::TS;
  for (int n = 0; n < 2; ++n)
    for (int k = 0; k < 3; ++k) {
      const bool real = n < NETS && k >= 1 && k < F::NL;
      y.h[n][k] = real ? TP::H(n, k) : -1;
      y.gpre[n][k] = real ? TP::Gpre(n, k) : -1;
    }
  for (int k = 0; k < 3; ++k) {
    y.hw[k] = k >= 1 && k < F::NL ? TP::HW(k) : 0;
    y.gpw[k] = k >= 1 && k < F::NL ? TP::GP(k) : 0;
  }
  for (int n = 0; n < 2; ++n) y.glast[n] = n < NETS ? TP::Glast(n) : -1;
  return y;
}
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
    CNF_G16(D, H1, H2)::bbefore(2)},                                                          \
   {k_wtrain16_fwd<D, H1, H2, 1>, k_wtrain16_fwd<D, H1, H2, 2>},                              \
   {k_wtrain16_bwd<D, H1, H2, 1>, k_wtrain16_bwd<D, H1, H2, 2>},                              \
   CNF_G16T(D, H1, H2)::NA,                                                                   \
   {CNF_G16T(D, H1, H2)::ks(0), CNF_G16T(D, H1, H2)::ks(1), CNF_G16T(D, H1, H2)::ks(2)},      \
   {CNF_G16T(D, H1, H2)::mt(0), CNF_G16T(D, H1, H2)::mt(1), CNF_G16T(D, H1, H2)::mt(2)},      \
   {64 * CNF_G16T(D, H1, H2)::sbefore(0), 64 * CNF_G16T(D, H1, H2)::sbefore(1),               \
    64 * CNF_G16T(D, H1, H2)::sbefore(2)},                                                    \
   {train_layout<D, H1, H2, 1>(), train_layout<D, H1, H2, 2>()}}

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

size_t w16_lds(const Shape& s, int rows = kRows) {
  return (size_t)kWaves * (rows * (s.D | 1) + s.D) * 4;
}

}  // namespace

// per layer: the forward stream and biases (all layers first), then the
// transposed stream of the reverse sweep (after the L forward records)
// transposed-stream floats per layer (pads included: G16T::lsp)
// forward A-stream floats per layer (pads included: G16::lsp)
static int64_t w16_la(const WEntry16* e, int nets) {
  const int ls = nets * (e->na / 64);
  return (int64_t)pad_fwd(ls) * 64;
}

static int64_t w16_lt(const WEntry16* e, int nets) {
  const int ls = nets * (e->nat / 64);
  return (int64_t)pad_ls(ls, CNF_W16_BWD_P16) * 64;
}

int64_t wide16_layer_floats(const Shape& s) {
  const WEntry16* e = w16find(s);
  return e ? w16_la(e, s.nets) + (int64_t)s.nets * e->nb + w16_lt(e, s.nets) : 0;
}

int wide16_prepare(const Shape& s, const float* const* params, void* prepared, hipStream_t st) {
  const WEntry16* e = w16find(s);
  if (!e) return CNF_OK;
  float* region = reinterpret_cast<float*>(static_cast<char*>(prepared) + idx_bytes(s)) +
                  s.wide_region;
  const int64_t LA = w16_la(e, s.nets), LF = LA + (int64_t)s.nets * e->nb;
  const int64_t LT = w16_lt(e, s.nets);
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
        g.abase = (int64_t)l * LF;
        g.adst = g.abase + (int64_t)pos * e->na + e->abefore[i];
        g.bdst = (int64_t)l * LF + LA + (int64_t)pos * e->nb + e->bbefore[i];
      }
    }
    // the reverse sweep's stream: s-net first (natural net order), each net's
    // Linears last first
    for (int net = 0; net < s.nets; ++net)
      for (int i = 0; i < s.n_lin; ++i) {
        const WSeg16& f = a.seg[net * s.n_lin + i];
        WSeg16& g = a.seg[a.nseg++];
        g = f;
        const int r = s.n_lin - 1 - i;  // reverse step of Linear i
        g.trans = 1;
        g.nin = f.nout;
        g.nout = f.nin;
        g.nm = e->mtT[r];
        g.nk = e->ksT[r];
        g.abase = (int64_t)s.L * LF + (int64_t)l * LT;
        g.adst = g.abase + (int64_t)net * e->nat + e->abeforeT[r];
        g.bdst = -1;
      }
    hipLaunchKernelGGL(k_prepare_wide16, dim3(a.nseg, 8), dim3(256), 0, st, a, region);
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
  const int64_t rows_per_block = (int64_t)kRunRows * kWaves;
  const dim3 grid((unsigned)((B + rows_per_block - 1) / rows_per_block)), block(64 * kWaves);
  WFn fn = e->fn[s.nets - 1][log_priors ? 2 : (inverse ? 1 : 0)];
  const size_t lds = CNF_W16_LDSA ? (size_t)(cdiv(kWaves * (kRunRows * (s.D | 1) + s.D), 64) * 64 + 2 * kAC * 64) * 4
                                  : w16_lds(s, kRunRows);
  hipLaunchKernelGGL(fn, grid, block, lds, st, W, inverse ? inv_q : fwd_q, in, out, ld, B,
                     s.L, log_priors);
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    set_hip_error(err);
    return CNF_ERR_HIP;
  }
  return CNF_OK;
}

int wide16_train_layout(const Shape& s, WTrain16Layout* out) {
  const WEntry16* e = w16find(s);
  if (!e || s.nets < 1 || s.nets > 2) return CNF_ERR_UNSUPPORTED;
  *out = e->lay[s.nets - 1];
  return CNF_OK;
}

int wide16_train_forward(const Shape& s, const void* prepared, const float* x, float* zst, int Cp,
                         int Dp, float* ld, float* tape, uint32_t* tbits, int64_t B,
                         const WSeed16* seed, hipStream_t st) {
  const WEntry16* e = w16find(s);
  if (!e || s.nets < 1 || s.nets > 2) return CNF_ERR_UNSUPPORTED;
  const char* base = static_cast<const char*>(prepared);
  const int32_t* fwd_q = reinterpret_cast<const int32_t*>(base);
  const float* W = reinterpret_cast<const float*>(base + idx_bytes(s)) + s.wide_region;
  const int64_t rows_per_block = (int64_t)kRows * kWaves;
  const dim3 grid((unsigned)((B + rows_per_block - 1) / rows_per_block)), block(64 * kWaves);
  SeedArgs sa{};
  sa.kind = -1;
  if (seed) {
    sa.y = seed->y;
    sa.G = seed->G;
    sa.gld = seed->gld;
    sa.part = seed->part;
    sa.det = seed->det;
    sa.grad_scale = seed->grad_scale;
    sa.kind = seed->kind;
  }
  const size_t lds = CNF_W16_TRAIN_LDSA && kRunRows == kRows
                         ? (size_t)(cdiv(kWaves * (kRows * (s.D | 1) + s.D), 64) * 64 + 2 * kAC * 64) * 4
                         : w16_lds(s);
  hipLaunchKernelGGL(e->tfwd[s.nets - 1], grid, block, lds, st, W, fwd_q, x, zst, ld, tape,
                     tbits, B, s.L, Cp, Dp, sa);
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    set_hip_error(err);
    return CNF_ERR_HIP;
  }
  return CNF_OK;
}

int wide16_train_backward(const Shape& s, const void* prepared, const float* gz,
                          const float* gz_all, float* dx, const float* gld, const float* tape,
                          const uint32_t* tbits, float* gbuf, int64_t B, hipStream_t st) {
  const WEntry16* e = w16find(s);
  if (!e || s.nets < 1 || s.nets > 2) return CNF_ERR_UNSUPPORTED;
  const char* base = static_cast<const char*>(prepared);
  const int32_t* inv_q = reinterpret_cast<const int32_t*>(base) + s.L * s.D;
  const float* W = reinterpret_cast<const float*>(base + idx_bytes(s)) + s.wide_region;
  const int64_t LF = w16_la(e, s.nets) + (int64_t)s.nets * e->nb;
  const int64_t rows_per_block = (int64_t)kRows * kWaves;
  const dim3 grid((unsigned)((B + rows_per_block - 1) / rows_per_block)), block(64 * kWaves);
  hipLaunchKernelGGL(e->tbwd[s.nets - 1], grid, block, w16_lds(s), st, W + s.L * LF, inv_q, gz,
                     gz_all, dx, gld, tape, tbits, gbuf, B, s.L);
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    set_hip_error(err);
    return CNF_ERR_HIP;
  }
  return CNF_OK;
}

}  // namespace cnf
