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

#include <cstdlib>
#include <mutex>
#include <type_traits>
#include <unordered_map>

#include "cnf_internal.h"
#include "cnf_valu_common.h"
#include "cnf_valu_io.h"

namespace cnf {
namespace {

using namespace valu;


// Fused L-layer coupling pass.  One block = ROWS threads = ROWS*RW logit
// vectors per tile.  PERSIST: a grid of (CUs x resident blocks) walks the
// tiles, prefetching the next tile's input into registers (16-B loads) while
// the current tile computes.
//
// Legacy alternate mask (alt, CNF_OPT_ALT_MASK; cnf_prepare reverses the odd
// layers' first-Linear columns and last-Linear rows): the flip-based stack then
// holds flip^(l+1) of the legacy layer-l output in logical order, i.e. the
// legacy output in RAW register order -- forward outputs are stored unflipped,
// and an inverse of an odd-L stack reads its input reversed (its every-layer
// outputs stay reversed).  SACT: the s-net's hidden activation (2: tanh).
template <int D, int H1, int H2, bool INV, bool STRICT, int RW, int ROWS, bool PERSIST, int WPE,
          bool FX, bool WL, bool WU = false, bool CH = false, bool DUP = false, int SACT = 1>
__global__ __launch_bounds__(ROWS, WPE) void k_valu(
    const float* __restrict__ Wg, const int32_t* __restrict__ qtab,
    const int32_t* __restrict__ lflag, const float* __restrict__ in, float* __restrict__ out,
    float* __restrict__ ld_out, float* __restrict__ all, int64_t B, int L, int scale, int shift,
    int any_perm, int vec_io, const int64_t* __restrict__ yl, float* __restrict__ loss_part,
    int kind, float det, int alt) {
  using T = typename RowT<RW>::type;
  constexpr int TR = ROWS * RW;  // rows per tile
  constexpr int TF = TR * D;     // floats per tile
  constexpr int NPT = (TF / 4 + ROWS - 1) / ROWS;  // prefetched float4 per thread
  // ONE dynamic LDS array: [tile: TF floats][weights (WL): L * layer_floats]
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sm = smem;
  const int tid = threadIdx.x;
  const bool vec = vec_io != 0;
  constexpr int NF = Net<D, H1, H2>::floats;
  const int layer_floats = (scale + shift) * NF;
  const float* W = Wg;
  if constexpr (WL) {
    // the whole weight blob, once per block, in one round trip of 16-B loads
    float* wl = smem + TF;
    const int n4 = (L * layer_floats) >> 2;  // layer_floats % 4 == 0 (compact layout)
    const float4* s4 = reinterpret_cast<const float4*>(Wg);
    float4* d4 = reinterpret_cast<float4*>(wl);
    if constexpr (DUP) {
      // each weight twice: the pair is the packed operand for the RW=2 rows
      for (int i = tid; i < n4; i += ROWS) {
        const float4 a = s4[i];
        d4[2 * i] = float4{a.x, a.x, a.y, a.y};
        d4[2 * i + 1] = float4{a.z, a.z, a.w, a.w};
      }
    } else {
      for (int i = tid; i < n4; i += ROWS) d4[i] = s4[i];
    }
    lds_barrier();
    W = wl;
  }
  using WP = typename std::conditional<DUP, f2, float>::type;
  const WP* WW = reinterpret_cast<const WP*>(W);
  const int64_t ntiles = (B + TR - 1) / TR;
  const int64_t nfull = B / TR;  // tiles whose TF floats are all in range
  const int64_t stride = PERSIST ? (int64_t)gridDim.x : ntiles;

  float4 pf[PERSIST ? NPT : 1];
  auto prefetch = [&](int64_t t) {
    const float4* s4 = reinterpret_cast<const float4*>(in + t * TF);
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const int k = i * ROWS + tid;
      if (k < TF / 4) pf[i] = s4[k];
    }
  };
  // WU: pull the weight blob into this XCD's L2 with one round trip of
  // vector loads, issued beside the first tile's input loads, so the first
  // waves' scalar-cache misses hit L2 instead of going to memory one Linear
  // at a time (the caches start cold at every dispatch).
  float4 wu[WU ? 4 : 1];
  constexpr int kWU = WU ? 4 : 0;
  if constexpr (WU) {
    const float4* s4 = reinterpret_cast<const float4*>(Wg);
    const int n4 = (L * layer_floats) >> 2;
#pragma unroll
    for (int i = 0; i < kWU; ++i) {
      const int k = tid + i * ROWS;
      wu[i] = k < n4 ? s4[k] : float4{0.f, 0.f, 0.f, 0.f};
    }
  }
  int64_t tile = blockIdx.x;
  if constexpr (PERSIST) {
    if (vec && tile < nfull) prefetch(tile);
  }
  float lt0 = 0.f, lt1 = 0.f, lt2 = 0.f;  // fused eval loss (calibrators.py:297-317)

  for (; tile < ntiles; tile += stride) {
    const int64_t row0 = tile * TR;
    const int nrows = (int)((B - row0) < TR ? (B - row0) : TR);
    lds_barrier();  // previous tile is done with sm
    bool from_regs = false;
    if constexpr (PERSIST) from_regs = vec && tile < nfull;
    if (from_regs) {
      float4* d4 = reinterpret_cast<float4*>(sm);
#pragma unroll
      for (int i = 0; i < NPT; ++i) {
        const int k = i * ROWS + tid;
        if (k < TF / 4) d4[k] = pf[i];
      }
    } else {
      tile_load<ROWS>(sm, in + row0 * D, nrows * D, vec);
    }
    int yv[RW];
    if (loss_part) load_labels<RW>(yl, row0, tid, ROWS, B, yv);
    lds_barrier();
    if constexpr (PERSIST) {
      const int64_t nt = tile + stride;
      if (vec && nt < nfull) prefetch(nt);  // lands while this tile computes
    }
    if constexpr (WU) {
#pragma unroll
      for (int i = 0; i < kWU; ++i) asm volatile("" ::"v"(wu[i].x));
    }
    // rows past the batch end read stale LDS: harmless, never stored
    T v[D];
    if (INV && alt && (L & 1)) {
#pragma unroll
      for (int k = 0; k < D; ++k) v[k] = get_row<ROWS>(sm, tid, D, D - 1 - k, T{});
    } else {
#pragma unroll
      for (int k = 0; k < D; ++k) v[k] = get_row<ROWS>(sm, tid, D, k, T{});
    }
    // every-layer store in orientation O (alt: the fixed raw orientation)
    auto st_all = [&](int i, auto O_) {
      constexpr bool O = decltype(O_)::value;
      float* dst = all + (int64_t)i * B * D + row0 * D;
      if (!alt) store_rows<D, ROWS, O>(dst, sm, v, nrows, vec);
      else if (INV && (L & 1)) store_rows<D, ROWS, true>(dst, sm, v, nrows, vec);
      else store_rows<D, ROWS, false>(dst, sm, v, nrows, vec);
    };

    T ld = splat(0.f, T{});
    // step index i = 0..L-1; layer = i (forward) or L-1-i (inverse)
    auto layer_of = [&](int i) { return INV ? L - 1 - i : i; };
    int i = 0;
    for (; i + 1 < L; i += 2) {
      int la = layer_of(i), lb = layer_of(i + 1);
      bool pa = any_perm && (lflag[la] & kFlagPerm), pb = any_perm && (lflag[lb] & kFlagPerm);
      step<D, H1, H2, INV, STRICT, false, FX && !STRICT, CH && !WL, SACT>(
          v, ld, WW + (int64_t)la * layer_floats, scale, shift, NF, pa, qtab + la * D);
      if (all) st_all(i, std::true_type{});
      step<D, H1, H2, INV, STRICT, true, FX && !STRICT, CH && !WL, SACT>(
          v, ld, WW + (int64_t)lb * layer_floats, scale, shift, NF, pb, qtab + lb * D);
      if (all) st_all(i + 1, std::false_type{});
    }
    bool odd = i < L;
    if (odd) {
      int la = layer_of(i);
      bool pa = any_perm && (lflag[la] & kFlagPerm);
      step<D, H1, H2, INV, STRICT, false, FX && !STRICT, CH && !WL, SACT>(
          v, ld, WW + (int64_t)la * layer_floats, scale, shift, NF, pa, qtab + la * D);
      if (all) st_all(i, std::true_type{});
    }
    // final orientation: odd L leaves the row reversed; the alt-mask forward
    // output is the raw register order
    const bool orev = odd && !(alt && !INV);
    if (out) {
      if (orev) store_rows<D, ROWS, true>(out + row0 * D, sm, v, nrows, vec);
      else store_rows<D, ROWS, false>(out + row0 * D, sm, v, nrows, vec);
    }
    if (ld_out) store_ld<ROWS>(ld_out, row0, tid, nrows, ld);
    if (loss_part) {
      if (orev) tile_loss<D, true>(v, ld, yv, kind, det, lt0, lt1, lt2);
      else tile_loss<D, false>(v, ld, yv, kind, det, lt0, lt1, lt2);
    }
  }
  if (loss_part) block_sum3<ROWS>(lt0, lt1, lt2, smem, loss_part);
}

// ---------------------------------------------------------------------------
// instantiation table
// ---------------------------------------------------------------------------
using KFn = void (*)(const float*, const int32_t*, const int32_t*, const float*, float*, float*,
                     float*, int64_t, int, int, int, int, int, const int64_t*, float*, int, float,
                     int);

struct Variant {
  KFn fn[2][2];  // [inverse][strict]
  int rw, rows, persist, wl;  // wl: 0 scalar weights, 1 LDS, 2 LDS pairs (DUP)
};

#define CNF_VARIANT_S(D, H1, H2, RW, ROWS, P, WPE, FX, WL, WU, CH, DUP, SA)                    \
  {{{k_valu<D, H1, H2, false, false, RW, ROWS, P, WPE, FX, WL, WU, CH, DUP, SA>,                \
     k_valu<D, H1, H2, false, true, RW, ROWS, P, WPE, FX, WL, WU, CH, DUP, SA>},                \
    {k_valu<D, H1, H2, true, false, RW, ROWS, P, WPE, FX, WL, WU, CH, DUP, SA>,                 \
     k_valu<D, H1, H2, true, true, RW, ROWS, P, WPE, FX, WL, WU, CH, DUP, SA>}},                \
   RW, ROWS, P, (WL) ? ((DUP) ? 2 : 1) : 0}
#define CNF_VARIANT_Y(D, H1, H2, RW, ROWS, P, WPE, FX, WL, WU, CH, DUP) \
  CNF_VARIANT_S(D, H1, H2, RW, ROWS, P, WPE, FX, WL, WU, CH, DUP, 1)
#define CNF_VARIANT_X(D, H1, H2, RW, ROWS, P, WPE, FX, WL, WU, CH) \
  CNF_VARIANT_Y(D, H1, H2, RW, ROWS, P, WPE, FX, WL, WU, CH, false)
#define CNF_VARIANT_U(D, H1, H2, RW, ROWS, P, WPE, FX, WL, WU) \
  CNF_VARIANT_X(D, H1, H2, RW, ROWS, P, WPE, FX, WL, WU, false)
#define CNF_VARIANT(D, H1, H2, RW, ROWS, P, WPE, FX, WL) \
  CNF_VARIANT_U(D, H1, H2, RW, ROWS, P, WPE, FX, WL, false)

struct Entry {
  int D, H1, H2;
  Variant small, large;  // dispatch on batch size (kLargeBatch)
  int nf;  // compact floats per net, must equal Shape::valu_net_floats
};

// Measured on MI355X (tools/bench_variants.py, tools/bench_scaling.py): up to
// a few M vectors the launch is latency-bound (few waves per SIMD for the
// whole kernel), where 2 vectors per lane with the weights staged once per
// block in LDS is fastest; past that the scalar-operand variant with one
// vector per lane sustains the higher rate.
constexpr int64_t kLargeBatch = 4ll << 20;

// Shipped configuration per shape: one vector per lane, 256-row tiles.
#define CNF_VALU(D, H1, H2)                                                     \
  {D, H1, H2, CNF_VARIANT(D, H1, H2, 2, 256, false, 4, true, true),             \
   CNF_VARIANT(D, H1, H2, 1, 256, false, 6, true, false), Net<D, H1, H2>::floats}

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

// Legacy tanh s-net shapes (CNF_OPT_S_TANH; code-old/realNVP.py:61 with its
// default hidden_size = [dim], and the reference default [5,5]): the same
// shipped configuration with the s-net's hidden layers on tanhf.
#define CNF_VALU_TANH(D, H1, H2)                                                          \
  {D, H1, H2, CNF_VARIANT_S(D, H1, H2, 2, 256, false, 4, true, true, false, false, false, 2), \
   CNF_VARIANT_S(D, H1, H2, 1, 256, false, 6, true, false, false, false, false, 2),            \
   Net<D, H1, H2>::floats}

const Entry kLTable[] = {
    CNF_VALU_TANH(3, 3, 0), CNF_VALU_TANH(10, 10, 0), CNF_VALU_TANH(10, 5, 5),
};
constexpr int kLBase = 1000;  // valu_id of kLTable[i] is kLBase + i

const Entry& entry_of(const Shape& s) {
  return s.valu_id >= kLBase ? kLTable[s.valu_id - kLBase] : kTable[s.valu_id];
}

int cu_count() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return v > 0 ? v : 256;
  }();
  return n;
}

int resident_blocks(KFn fn, int threads) {
  static std::mutex mu;
  static std::unordered_map<const void*, int> cache;
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find((const void*)fn);
  if (it != cache.end()) return it->second;
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, threads, 0) != hipSuccess || n < 1)
    n = 1;
  cache[(const void*)fn] = n;
  return n;
}

}  // namespace

int valu_supported(const Shape& s) {
  int h1 = s.n_lin >= 2 ? s.units[1] : 0;
  int h2 = s.n_lin >= 3 ? s.units[2] : 0;
  if (s.n_lin > 3) return -1;
  if (s.s_tanh && s.scale) {
    for (int i = 0; i < (int)(sizeof(kLTable) / sizeof(kLTable[0])); ++i)
      if (kLTable[i].D == s.D && kLTable[i].H1 == h1 && kLTable[i].H2 == h2) return kLBase + i;
    return -1;
  }
  for (int i = 0; i < (int)(sizeof(kTable) / sizeof(kTable[0])); ++i)
    if (kTable[i].D == s.D && kTable[i].H1 == h1 && kTable[i].H2 == h2) return i;
  return -1;
}

static const Variant* pick_variant(const Shape& s, int64_t B) {
  const Entry& e = entry_of(s);
  const bool lds_fits =
      (size_t)256 * 2 * s.D * 4 + (size_t)s.L * s.nets * s.valu_net_floats * 4 <= 64 * 1024;
  return (B > kLargeBatch || !lds_fits) ? &e.large : &e.small;
}

static int64_t blocks_for(const Shape& s, const Variant* var, KFn fn, int64_t B) {
  const int64_t tr = (int64_t)var->rows * var->rw;
  int64_t nblk = (B + tr - 1) / tr;
  if (var->persist) {
    const int64_t cap = (int64_t)cu_count() * resident_blocks(fn, var->rows);
    if (nblk > cap) nblk = cap;
  }
  return nblk;
}

// Loss partial records a fused eval may write: whichever of k_sgpr / k_valu
// serves the launch (k_valu takes misaligned views and permuted stacks).
int valu_loss_blocks(const Shape& s, int64_t B) {
  if (s.valu_id < 0) return -1;
  const Variant* var = pick_variant(s, B);
  int64_t n = blocks_for(s, var, var->fn[0][s.strict ? 1 : 0], B);
  if (sgpr_enabled(s)) {
    const int64_t m = sgpr_blocks(s, B);
    if (m > n) n = m;
  }
  return (int)n;
}

int valu_run(const Shape& s, const void* prepared, const float* in, float* out, float* ld,
             float* all, int64_t B, bool inverse, hipStream_t st, const int64_t* y,
             float* loss_ws, int kind, float det, float* loss_terms) {
  if (s.valu_id < 0) return CNF_ERR_UNSUPPORTED;
  if (B == 0) return CNF_OK;
  // every-layer outputs (all != null) stay on k_valu: its LDS-staged stores
  // write the L*B*D floats at ~4.2 TB/s, k_sgpr's per-lane ones at ~3 TB/s
  if (sgpr_enabled(s) && all == nullptr) {
    const int r = sgpr_run(s, prepared, in, out, ld, all, B, inverse, st, y, loss_ws, kind, det,
                           loss_terms);
    if (r != CNF_ERR_UNSUPPORTED) return r;
  }
  const Entry& e = entry_of(s);
  if (e.nf != s.valu_net_floats) return CNF_ERR_DESC;  // host/device layout disagree
  const Variant* var = pick_variant(s, B);
  const char* base = static_cast<const char*>(prepared);
  const int32_t* fwd_q = reinterpret_cast<const int32_t*>(base);
  const int32_t* inv_q = fwd_q + s.L * s.D;
  const int32_t* flags = inv_q + s.L * s.D;
  const float* W = reinterpret_cast<const float*>(base + idx_bytes(s));
  auto al = [](const void* p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  int vec = al(in) && al(out) && al(all);
  KFn fn = var->fn[inverse ? 1 : 0][s.strict ? 1 : 0];
  const int64_t tr = (int64_t)var->rows * var->rw;
  const int64_t nblk = blocks_for(s, var, fn, B);
  size_t lds = (size_t)tr * s.D * 4;
  if (lds < (size_t)3 * var->rows * 4 + 4 * 65) lds = (size_t)3 * var->rows * 4 + 4 * 65;
  if (var->wl) lds += (size_t)s.L * s.nets * s.valu_net_floats * 4 * var->wl;
  if (lds > 160 * 1024) return CNF_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(fn, dim3((unsigned)nblk), dim3(var->rows), lds, st, W,
                     inverse ? inv_q : fwd_q, flags, in, out, ld, all, B, s.L, s.scale, s.shift,
                     s.any_perm ? 1 : 0, vec, y, loss_ws ? loss_ws + 4 : nullptr, kind, det,
                     s.alt_mask ? 1 : 0);
  if (loss_ws) reduce_partials(loss_ws + 4, (int)nblk, 4, 0, nullptr, loss_terms, st);
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    set_hip_error(err);
    return CNF_ERR_HIP;
  }
  return CNF_OK;
}

}  // namespace cnf
