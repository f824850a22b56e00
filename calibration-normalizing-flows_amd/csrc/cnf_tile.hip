// General-shape coupling kernel on the f32 matrix cores (MFMA).
//
// Serves every NvpCouplingLayer stack the narrow VALU kernel does not: wide
// logit vectors (CIFAR-100: D=100, hidden_size=[100,100]), any number of
// hidden layers, any widths up to CNF_MAX_WIDTH.  One wave owns 16 logit
// vectors for the whole L-layer stack; its activations live in LDS laid out
// feature-major ([feature][16 vectors]), which is exactly the B-operand layout
// of v_mfma_f32_16x16x4_f32 (lane l reads B[k = l>>4][j = l&15]), so each
// Linear is a chain of MFMAs whose A operand is a pre-tiled, coalesced 256-B
// slice of the weights (one per lane per MFMA, prepared by cnf_prepare).
// f32-in/f32-acc MFMA is an exact fmaf chain -- no reduced precision.
//
// Per layer (flows/flows.py:101-126): s-net and t-net on the conditioning half
// (mask-reduced K), fused bias + ReLU epilogues (flows/utils.py:26-31), the
// affine update and the log-det partial sums in registers, then the flip /
// random permutation as an LDS gather through the layer's index table.
#include <hip/hip_runtime.h>

#include "cnf_internal.h"

namespace cnf {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kWaves = 4;  // max waves (16-vector tiles) per block
constexpr int kTileRows = 16;

struct TileArgs {
  int D, DT, DC, NO, L, n_lin, scale, shift;
  int s_act;                 // s-net hidden activation: 1 ReLU, 2 tanh (CNF_OPT_S_TANH)
  int nout[kMaxLin], OT[kMaxLin], KS[kMaxLin];
  int64_t lin_off[kMaxLin];  // float offset of linear i inside a tiled net
  int64_t net_floats, layer_floats;
  int Dp, Hp, NOp;           // LDS rows of X, activation and S/T buffers
  int wave_floats;           // LDS floats per wave
};

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <bool STRICT>
__device__ __forceinline__ float relu(float a) {
  if constexpr (STRICT) return a < 0.f ? 0.f : a;
  else return fmaxf(a, 0.f);
}

// act: 0 none (a net's last Linear), 1 ReLU, 2 tanh (legacy s-net)
template <bool STRICT>
__device__ __forceinline__ void epilogue(const floatx4& acc, int ot, const float* __restrict__ bias,
                                         float* OUT, int nout, int act, float p0, int lane) {
  const int c = lane & 15, g = lane >> 4;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int o = ot * 16 + 4 * g + r;
    float v = acc[r] + bias[o] + p0;
    if (act == 1) v = relu<STRICT>(v);
    else if (act == 2) v = tanhf(v);
    OUT[o * kTileRows + c] = o < nout ? v : 0.f;
  }
}

// OUT[o][j] = act(bias[o] + sum_k W[o][k] * IN[k][j]) for o < OT*16, j < 16.
template <bool STRICT>
__device__ __forceinline__ void gemm(const float* __restrict__ lin, const float* IN, float* OUT,
                                     int OT, int KS, int nout, int act, float p0, int lane) {
  const float* __restrict__ bias = lin;
  const float* __restrict__ tiles = lin + OT * 16;
  const int boff = (lane >> 4) * kTileRows + (lane & 15);
  for (int ot = 0; ot < OT; ot += 2) {
    const bool two = ot + 1 < OT;
    floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    const float* __restrict__ w0 = tiles + (int64_t)ot * KS * 64 + lane;
    const float* __restrict__ w1 = w0 + KS * 64;
    if (two) {
#pragma unroll 4
      for (int ks = 0; ks < KS; ++ks) {
        const float b = IN[ks * 4 * kTileRows + boff];
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(w0[ks * 64], b, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(w1[ks * 64], b, acc1, 0, 0, 0);
      }
    } else {
      for (int ks = 0; ks < KS; ++ks) {
        const float b = IN[ks * 4 * kTileRows + boff];
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(w0[ks * 64], b, acc0, 0, 0, 0);
      }
    }
    epilogue<STRICT>(acc0, ot, bias, OUT, nout, act, p0, lane);
    if (two) epilogue<STRICT>(acc1, ot + 1, bias, OUT, nout, act, p0, lane);
  }
}

// One conditioner MLP: conditioning rows of X -> OUT rows [0, NO).
template <bool STRICT>
__device__ __forceinline__ void mlp(const TileArgs& a, const float* __restrict__ net,
                                    const float* Xc, float* A0, float* A1, float* OUT, float p0,
                                    int lane, int act) {
  const float* in = Xc;
  for (int i = 0; i < a.n_lin; ++i) {
    const bool last = i == a.n_lin - 1;
    float* o = last ? OUT : ((i & 1) ? A1 : A0);
    gemm<STRICT>(net + a.lin_off[i], in, o, a.OT[i], a.KS[i], a.nout[i], last ? 0 : act,
                 i == 0 ? p0 : 0.f, lane);
    wave_sync();
    in = o;
  }
}

template <bool INV, bool STRICT>
__global__ __launch_bounds__(256) void k_tile(TileArgs a, const float* __restrict__ W,
                                              const int32_t* __restrict__ qtab,
                                              const float* __restrict__ in,
                                              float* __restrict__ out, float* __restrict__ ld_out,
                                              float* __restrict__ all, int64_t B) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nw = blockDim.x >> 6;
  const int64_t row0 = ((int64_t)blockIdx.x * nw + wave) * kTileRows;
  if (row0 >= B) return;  // only wave-local synchronisation below
  const int nrows = (int)((B - row0) < kTileRows ? (B - row0) : kTileRows);
  const int D = a.D, DT = a.DT;
  float* X = smem + (int64_t)wave * a.wave_floats;
  float* Xn = X + a.Dp * kTileRows;
  float* A0 = Xn + a.Dp * kTileRows;
  float* A1 = A0 + a.Hp * kTileRows;
  float* S = A1 + a.Hp * kTileRows;
  float* T = S + a.NOp * kTileRows;
  const int c = lane & 15;

  for (int i = D * kTileRows + lane; i < a.Dp * kTileRows; i += 64) X[i] = Xn[i] = 0.f;
  const float* src = in + row0 * D;
  for (int i = lane; i < kTileRows * D; i += 64) {
    const int r = i / D, f = i - r * D;
    X[f * kTileRows + r] = r < nrows ? src[i] : 0.f;
  }
  wave_sync();

  float ld = 0.f;
  for (int st = 0; st < a.L; ++st) {
    const int l = INV ? a.L - 1 - st : st;
    const int32_t* __restrict__ q = qtab + l * D;
    if constexpr (INV) {  // z.flip(1) then z[:, rev_perm]  (flows/flows.py:115-117)
      for (int i = lane; i < D * kTileRows; i += 64) {
        const int j = i >> 4;
        Xn[i] = X[q[j] * kTileRows + (i & 15)];
      }
      wave_sync();
      float* t = X; X = Xn; Xn = t;
    }
    float p0 = 0.f;
    if constexpr (STRICT) {
      for (int j = 0; j < DT; ++j) p0 += 0.f * X[j * kTileRows + c];
    }
    const float* __restrict__ wl = W + (int64_t)l * a.layer_floats;
    if (a.scale) {
      mlp<STRICT>(a, wl, X + DT * kTileRows, A0, A1, S, p0, lane, a.s_act);
      wl += a.net_floats;
    }
    if (a.shift) mlp<STRICT>(a, wl, X + DT * kTileRows, A0, A1, T, p0, lane, 1);
    const int nupd = STRICT ? D : DT;
    for (int i = lane; i < nupd * kTileRows; i += 64) {
      const int j = i >> 4;
      const float x = X[i];
      const float s = a.scale ? S[i] : 0.f;
      const float t = a.shift ? T[i] : 0.f;
      float y = INV ? (x - t) * expf(-s) : fmaf(x, expf(s), t);
      if (j < DT) {
        X[i] = STRICT ? 0.f * x + y : y;
        ld += INV ? -s : s;
      } else {  // STRICT only: masked position keeps x unless exp overflowed
        X[i] = x + 0.f * y;
        ld += 0.f * s;
      }
    }
    wave_sync();
    if constexpr (!INV) {  // z[:, perm] then z.flip(1)  (flows/flows.py:110-112)
      for (int i = lane; i < D * kTileRows; i += 64) {
        const int j = i >> 4;
        Xn[i] = X[q[j] * kTileRows + (i & 15)];
      }
      wave_sync();
      float* t = X; X = Xn; Xn = t;
    }
    if (all) {
      float* dst = all + (int64_t)st * B * D + row0 * D;
      for (int i = lane; i < nrows * D; i += 64) {
        const int r = i / D, f = i - r * D;
        dst[i] = X[f * kTileRows + r];
      }
    }
  }
  if (out) {
    float* dst = out + row0 * D;
    for (int i = lane; i < nrows * D; i += 64) {
      const int r = i / D, f = i - r * D;
      dst[i] = X[f * kTileRows + r];
    }
  }
  ld += __shfl_xor(ld, 16);
  ld += __shfl_xor(ld, 32);
  if (ld_out && lane < nrows) ld_out[row0 + lane] = ld;
}

TileArgs make_args(const Shape& s) {
  TileArgs a{};
  a.D = s.D; a.DT = s.DT; a.DC = s.DC; a.NO = s.NO; a.L = s.L; a.n_lin = s.n_lin;
  a.scale = s.scale; a.shift = s.shift;
  a.s_act = s.s_tanh ? 2 : 1;
  for (int i = 0; i < s.n_lin; ++i) {
    a.nout[i] = s.lin_nout[i];
    a.OT[i] = s.lin_OT[i];
    a.KS[i] = s.lin_KS[i];
    a.lin_off[i] = s.tile_lin_off[i];
  }
  a.net_floats = s.tile_net_floats;
  a.layer_floats = s.tile_layer_floats;
  a.Dp = (s.D + 3) / 4 * 4 + 4;
  a.Hp = s.tile_hp;
  a.NOp = s.tile_nop;
  a.wave_floats = (2 * a.Dp + 2 * a.Hp + 2 * a.NOp) * kTileRows;
  return a;
}

// ---------------------------------------------------------------------------
// cnf_prepare: one launch per layer; the parameter pointers and the layer's
// index tables travel by value in the kernel arguments (no host staging).
// ---------------------------------------------------------------------------
struct PrepSeg {
  const float* W;
  const float* b;
  int64_t dst;  // float offset in the weights region
  float wmul, bmul;  // mode 3: weights / bias scale (relu clamp 2^-64, log2 e; cnf_sgpr.hip)
  int16_t mode;      // 0: natural copy, 1: MFMA tiles, 2: compact (VALU), 3: packed (SGPR)
  int16_t nout_full, nin_full, in_off, nin, nout, OT, KS;
  int16_t rev_in, rev_out;  // legacy alternate mask, odd layer: input columns / output rows reversed
};

// cnf_prepare's work as few launches as the kernel-argument budget allows:
// every (layer, net, Linear, layout copy) segment is one block of k_prepare
// (up to kPrepJobs per launch, < 4 KB of arguments), and one k_prep_idx
// launch writes the gather tables of as many layers as fit.  (Round 2 made
// four launches per layer: 20 per prepare of the calibrator's 5-layer flow,
// re-run after every optimizer step.)
constexpr int kPrepJobs = 60;
struct PrepBatch {
  PrepSeg seg[kPrepJobs];
  int nseg;
};
constexpr int kPrepIdxInts = 900;
struct PrepIdx {
  int32_t v[kPrepIdxInts];  // per layer: fq[D], iq[D], flag
  int D, L, l0, nl;
};

__global__ void k_prep_idx(PrepIdx a, int32_t* __restrict__ idx) {
  const int per = 2 * a.D + 1;
  for (int i = threadIdx.x; i < a.nl * per; i += blockDim.x) {
    const int l = a.l0 + i / per, j = i % per;
    const int32_t v = a.v[i];
    if (j < a.D) idx[l * a.D + j] = v;
    else if (j < 2 * a.D) idx[a.L * a.D + l * a.D + (j - a.D)] = v;
    else idx[2 * a.L * a.D + l] = v;
  }
}

__global__ void k_prepare(PrepBatch a, float* __restrict__ wreg) {
  const PrepSeg& g = a.seg[blockIdx.x];
  float* dst = wreg + g.dst;
  auto orow = [&](int o) { return g.rev_out ? g.nout_full - 1 - o : o; };
  auto icol = [&](int c) { return g.rev_in ? g.nin_full - 1 - c : c; };
  if (g.mode == 0) {
    const int64_t nW = (int64_t)g.nout_full * g.nin_full;
    for (int64_t i = threadIdx.x; i < nW + g.nout_full; i += blockDim.x) {
      if (i < nW) {
        const int o = (int)(i / g.nin_full), c = (int)(i - (int64_t)o * g.nin_full);
        dst[i] = g.W[(int64_t)orow(o) * g.nin_full + icol(c)];
      } else {
        dst[i] = g.b[orow((int)(i - nW))];
      }
    }
    return;
  }
  if (g.mode == 3) {  // rows [w_o0, b_o, w_o1 .. w_o(nin-1)] at even stride, zero padded
    const int S = (g.nin + 2) & ~1;
    const int64_t n = ((int64_t)g.nout * S + 15) & ~15;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
      float v = 0.f;
      const int o = (int)(i / S), j = (int)(i - (int64_t)o * S);
      if (o < g.nout) {
        if (j == 1) v = g.b[o] * g.bmul;
        else if (j == 0 || j <= g.nin) {
          const int k = j == 0 ? 0 : j - 1;
          v = g.W[(int64_t)o * g.nin_full + g.in_off + k] * g.wmul;
        }
      }
      dst[i] = v;
    }
    return;
  }
  if (g.mode == 2) {
    const int S = (g.nin + 3) & ~3, NP = (g.nout_full + 3) & ~3;
    const int64_t nW = (int64_t)g.nout_full * S;
    for (int64_t i = threadIdx.x; i < nW + NP; i += blockDim.x) {
      float v = 0.f;
      if (i < nW) {
        const int o = (int)(i / S), k = (int)(i - (int64_t)o * S);
        if (k < g.nin) v = g.W[(int64_t)orow(o) * g.nin_full + icol(g.in_off + k)];
      } else if (i - nW < g.nout_full) {
        v = g.b[orow((int)(i - nW))];
      }
      dst[i] = v;
    }
    return;
  }
  for (int o = threadIdx.x; o < g.OT * 16; o += blockDim.x) dst[o] = o < g.nout ? g.b[orow(o)] : 0.f;
  const int64_t ntile = (int64_t)g.OT * g.KS * 64;
  float* tiles = dst + g.OT * 16;
  for (int64_t e = threadIdx.x; e < ntile; e += blockDim.x) {
    const int64_t ot = e / (g.KS * 64);
    const int rem = (int)(e - ot * g.KS * 64);
    const int ks = rem >> 6, ln = rem & 63;
    const int o = (int)ot * 16 + (ln & 15), k = ks * 4 + (ln >> 4);
    tiles[e] = (o < g.nout && k < g.nin)
                   ? g.W[(int64_t)orow(o) * g.nin_full + icol(g.in_off + k)] : 0.f;
  }
}

}  // namespace

int tile_configure(Shape* s) {
  s->NO = s->strict ? s->D : s->DT;
  int hp = 16;
  int64_t off = 0;
  for (int i = 0; i < s->n_lin; ++i) {
    const int nin_full = s->units[i], nout_full = s->units[i + 1];
    const bool first = i == 0, last = i == s->n_lin - 1;
    const int nin = first ? s->DC : nin_full;
    const int nout = last ? s->NO : nout_full;
    s->lin_nin[i] = nin;
    s->lin_nout[i] = nout;
    s->lin_inoff[i] = first ? s->DT : 0;
    s->lin_OT[i] = (nout + 15) / 16;
    s->lin_KS[i] = (nin + 3) / 4;
    s->tile_lin_off[i] = off;
    off += (int64_t)s->lin_OT[i] * 16 + (int64_t)s->lin_OT[i] * s->lin_KS[i] * 64;
    if (!last && s->lin_OT[i] * 16 > hp) hp = s->lin_OT[i] * 16;
    if (nout_full > CNF_MAX_WIDTH || nin_full > CNF_MAX_WIDTH) return CNF_ERR_UNSUPPORTED;
  }
  s->tile_net_floats = off;
  s->tile_layer_floats = off * s->nets;
  s->tile_hp = hp;
  s->tile_nop = (s->NO + 15) / 16 * 16;
  const int dp = (s->D + 3) / 4 * 4 + 4;
  const size_t per_wave = (size_t)(2 * dp + 2 * hp + 2 * s->tile_nop) * kTileRows * 4;
  int waves = (int)((160 * 1024) / per_wave);
  if (waves < 1) return CNF_ERR_UNSUPPORTED;
  if (waves > kWaves) waves = kWaves;
  s->tile_waves = waves;
  s->tile_lds_bytes = per_wave * waves;
  s->wide_region = s->tile_layer_floats * s->L;
  s->wide_floats = wide_layer_floats(*s) * s->L;
  s->plain_region = s->wide_region + s->wide_floats;
  return CNF_OK;
}

int tile_run(const Shape& s, const void* prepared, const float* in, float* out, float* ld,
             float* all, int64_t B, bool inverse, hipStream_t st) {
  if (B == 0) return CNF_OK;
  if (!all && s.wide_floats > 0 && wide_ok(s))
    return wide_run(s, prepared, in, out, ld, B, inverse, st);
  TileArgs a = make_args(s);
  const char* base = static_cast<const char*>(prepared);
  const int32_t* fwd_q = reinterpret_cast<const int32_t*>(base);
  const int32_t* inv_q = fwd_q + s.L * s.D;
  const float* W = reinterpret_cast<const float*>(base + idx_bytes(s));
  const int64_t vecs_per_block = (int64_t)s.tile_waves * kTileRows;
  dim3 grid((unsigned)((B + vecs_per_block - 1) / vecs_per_block)), block(64 * s.tile_waves);
  auto fn = inverse ? (s.strict ? k_tile<true, true> : k_tile<true, false>)
                    : (s.strict ? k_tile<false, true> : k_tile<false, false>);
  hipLaunchKernelGGL(fn, grid, block, s.tile_lds_bytes, st, a, W, inverse ? inv_q : fwd_q, in, out,
                     ld, all, B);
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    set_hip_error(err);
    return CNF_ERR_HIP;
  }
  return CNF_OK;
}

int prepare_run(const Shape& s, const float* const* params, void* prepared, hipStream_t st) {
  char* base = static_cast<char*>(prepared);
  int32_t* idx = reinterpret_cast<int32_t*>(base);
  float* wreg = reinterpret_cast<float*>(base + idx_bytes(s));
  const bool tiled = s.family == Family::kTile;
  PrepBatch batch{};
  PrepIdx tab{};
  tab.D = s.D;
  tab.L = s.L;
  auto flush_jobs = [&]() {
    if (batch.nseg > 0)
      hipLaunchKernelGGL(k_prepare, dim3(batch.nseg), dim3(256), 0, st, batch, wreg);
    batch.nseg = 0;
  };
  auto push = [&](const PrepSeg& g) {
    if (batch.nseg == kPrepJobs) flush_jobs();
    batch.seg[batch.nseg++] = g;
  };
  auto flush_idx = [&]() {
    if (tab.nl > 0) hipLaunchKernelGGL(k_prep_idx, dim3(1), dim3(256), 0, st, tab, idx);
    tab.l0 += tab.nl;
    tab.nl = 0;
  };
  const int per = 2 * s.D + 1;
  int pi = 0;
  for (int l = 0; l < s.L; ++l) {
    PrepSeg segs[2 * kMaxLin];
    int nseg = 0;
    int64_t dst = tiled ? (int64_t)l * s.tile_layer_floats
                        : (int64_t)l * s.valu_net_floats * s.nets;
    for (int net = 0; net < s.nets; ++net) {
      for (int i = 0; i < s.n_lin; ++i) {
        PrepSeg& g = segs[nseg++];
        g = PrepSeg{};
        g.W = params[pi++];
        g.b = params[pi++];
        if (!g.W || !g.b) return CNF_ERR_NULL;
        g.nout_full = (int16_t)s.units[i + 1];
        g.nin_full = (int16_t)s.units[i];
        g.rev_in = g.rev_out = 0;
        g.wmul = g.bmul = 1.f;
        if (s.alt_mask && (l & 1)) {
          g.rev_in = i == 0;
          g.rev_out = i == s.n_lin - 1;
        }
        if (tiled) {
          g.mode = 1;
          g.in_off = (int16_t)s.lin_inoff[i];
          g.nin = (int16_t)s.lin_nin[i];
          g.nout = (int16_t)s.lin_nout[i];
          g.OT = (int16_t)s.lin_OT[i];
          g.KS = (int16_t)s.lin_KS[i];
          g.dst = dst + s.tile_lin_off[i];
        } else {
          g.mode = 2;
          g.in_off = (int16_t)(i == 0 ? s.DT : 0);
          g.nin = (int16_t)(i == 0 ? s.DC : g.nin_full);
          g.nout = g.nout_full;
          g.dst = dst + s.valu_lin_off[i];
        }
      }
      dst += tiled ? s.tile_net_floats : s.valu_net_floats;
    }
    for (int k = 0; k < nseg; ++k) push(segs[k]);
    {
      // natural copy of the layer (state_dict order) for the reverse mode
      int64_t d = s.plain_region + (int64_t)l * s.layer_floats;
      for (int k = 0; k < nseg; ++k) {
        PrepSeg g = segs[k];
        g.mode = 0;
        g.dst = d;
        d += (int64_t)g.nout_full * g.nin_full + g.nout_full;
        push(g);
      }
    }
    if (!tiled && s.sp_ok) {
      // second copy of the layer in the packed SGPR layout (no index block)
      const int64_t d2 = s.sp_region + (int64_t)l * s.sp_net_floats * s.nets;
      const int64_t d3 = s.vp_region + (int64_t)l * s.sp_net_floats * s.nets;
      for (int k = 0; k < nseg; ++k) {
        PrepSeg g = segs[k];
        const int i = k % s.n_lin;
        g.mode = 3;
        const bool last = i == s.n_lin - 1;
        g.nout = (int16_t)(last ? s.DT : g.nout_full);
        // k_sgpr folds relu into the clamp bit: hidden outputs are kept scaled
        // by 2^-64 (so relu(a) 2^-64 = clamp(a 2^-64, 0, 1)) and the next
        // Linear's input columns undo it; the s-net (first net when scale is
        // on) ends in log2(e) * s.  Powers of two: exact.
        const float sin = i == 0 ? 1.f : 0x1p-64f;
        float sout = last ? 1.f : 0x1p-64f;
        if (s.scale && k / s.n_lin == 0 && last) sout *= 1.4426950408889634f;
        g.wmul = sout / sin;
        g.bmul = sout;
        g.dst = d2 + (k / s.n_lin) * s.sp_net_floats + s.sp_lin_off[i];
        push(g);
        // ... and a plain copy (no relu or log2(e) scaling) for the reverse mode
        g.wmul = g.bmul = 1.f;
        g.dst = d3 + (k / s.n_lin) * s.sp_net_floats + s.sp_lin_off[i];
        push(g);
      }
    }
    // gather tables of layer l
    const int64_t* perm = nullptr;
    if (s.any_perm && s.perms_host) {
      const int64_t* p = s.perms_host + (int64_t)l * s.D;
      if (p[0] >= 0) perm = p;
    }
    int32_t flag = perm ? kFlagPerm : 0;
    int32_t rev[CNF_MAX_DIM];
    if (perm) {
      for (int j = 0; j < s.D; ++j) rev[perm[j]] = j;
    }
    // legacy alternate mask (no data flip): the flip-based stack with odd
    // layers' weights reversed computes flip^(l+1) of the legacy layer l
    // output, so an odd-L stack ends with one extra flip: its last table is
    // the identity
    const bool unflip = s.alt_mask && (s.L & 1) && l == s.L - 1;
    if (unflip) flag = kFlagPerm;
    if ((tab.nl + 1) * per > kPrepIdxInts) flush_idx();
    int32_t* v = tab.v + tab.nl * per;
    for (int j = 0; j < s.D; ++j) {
      // forward: out[j] = z[perm[D-1-j]]; inverse: x_in[j] = z[D-1-rev_perm[j]]
      v[j] = unflip ? j : (perm ? (int32_t)perm[s.D - 1 - j] : s.D - 1 - j);
      v[s.D + j] = unflip ? j : (perm ? s.D - 1 - rev[j] : s.D - 1 - j);
    }
    v[2 * s.D] = flag;
    ++tab.nl;
  }
  flush_jobs();
  flush_idx();
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    set_hip_error(err);
    return CNF_ERR_HIP;
  }
  if (tiled && s.wide_floats > 0) return wide_prepare(s, params, prepared, st);
  return CNF_OK;
}

}  // namespace cnf
