// Reverse mode of the fused coupling stack (training path).
//
// Replaces torch autograd through Flow.forward (flows/flows.py:17-25,
// NvpCouplingLayer.forward :101-112, MLP.forward flows/utils.py:26-31) and,
// fused with it, the calibrator loss of TorchFlowCalibrator.fit
// (calibrators.py:287-295) or the CE - det*mean(ld) loss of
// run_experiment3D.py:102-107.
//
// One wave = 64 logit vectors (one per lane) for the whole L-layer stack,
// grid-striding over the batch:
//   forward sweep   as cnf_forward, stashing each layer's transformed inputs
//                   x_T in LDS (the conditioning inputs pass through unchanged,
//                   so with the stash every intermediate is exact);
//   loss            log-softmax, per-row loss terms and dL/dz_L in registers;
//   backward sweep  per layer: undo flip/perm, recompute both conditioner MLPs
//                   on the conditioning half, back-propagate through the affine
//                   update and both MLPs (transpose products on scalar weights);
//   weight grads    dW = sum over rows of g (x) h is a GEMM over the batch: each
//                   net's gradient stack G = [g_h1, g_h2, g_out] and input stack
//                   H = [c, h1, h2, 1] are staged [feature][row] in LDS and
//                   folded into per-wave accumulator tiles by
//                   v_mfma_f32_16x16x4_f32 with the 64 rows as the K dimension.
// Per-block partial sums land in the workspace; a second kernel adds them in
// block order -- no float atomics, bit-reproducible run to run.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <unordered_map>
#include <type_traits>

#include "cnf_internal.h"
#include "cnf_valu_common.h"
#include "cnf_sgpr_common.h"
#include "cnf_valu_io.h"

namespace cnf {
namespace {

using namespace valu;
typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kVRows = 64;    // one wave per block, one vector per lane
constexpr int kVGrid = 2048;  // max blocks: fixed, so the reduction order is device-independent
constexpr int kGP = 65;       // staging row stride (floats): conflict-free [feature][row] writes
constexpr float kEps = 1e-7f; // calibrators.py:289

template <int D, int H1, int H2>
struct VS {
  static constexpr int DT = D / 2, DC = D - D / 2;
  static constexpr int NL = H1 == 0 ? 1 : (H2 == 0 ? 2 : 3);
  static constexpr int GS = H1 + H2 + DT;        // [g_h1, g_h2, g_out]
  static constexpr int HS = DC + H1 + H2 + 1;    // [c, h1, h2, 1]
  static constexpr int TG = (GS + 15) / 16, TH = (HS + 15) / 16;
  static constexpr int ACC = TG * TH * 256;      // accumulator floats per (layer, net)
  static constexpr int NFN = H1 == 0 ? D * D + D  // natural floats per net
                             : H2 == 0 ? H1 * D + H1 + D * H1 + D
                                       : H1 * D + H1 + H2 * H1 + H2 + D * H2 + D;
};

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One MLP forward keeping its activations (compact weights, cnf_valu_common.h).
template <int D, int H1, int H2>
__device__ __forceinline__ void mlp_keep(const float* __restrict__ w, const float* c, float* h1,
                                         float* h2, float* out) {
  constexpr int DT = D / 2, DC = D - D / 2;
  if constexpr (H1 == 0) {
    linear<DC, D, DT, false, false, false>(w, c, out, 0.f);
  } else if constexpr (H2 == 0) {
    linear<DC, H1, H1, true, false, false>(w, c, h1, 0.f);
    linear<H1, D, DT, false, false, false>(w + Lin<DC, H1>::floats, h1, out, 0.f);
  } else {
    linear<DC, H1, H1, true, false, false>(w, c, h1, 0.f);
    const float* w2 = w + Lin<DC, H1>::floats;
    linear<H1, H2, H2, true, false, false>(w2, h1, h2, 0.f);
    linear<H2, D, DT, false, false, false>(w2 + Lin<H1, H2>::floats, h2, out, 0.f);
  }
}

// Fold one net's (G, H) stacks of this wave's 64 rows into its accumulator.
template <int TG, int TH>
__device__ __forceinline__ void accumulate(float* acc, const float* Gs, const float* Hs,
                                           int lane) {
  const int c = lane & 15, g = lane >> 4;
#pragma unroll
  for (int tg = 0; tg < TG; ++tg) {
#pragma unroll
    for (int th = 0; th < TH; ++th) {
      float* base = acc + (tg * TH + th) * 256;
      floatx4 a4;
#pragma unroll
      for (int r = 0; r < 4; ++r) a4[r] = base[(4 * g + r) * 16 + c];
      const float* ga = Gs + (16 * tg + c) * kGP + g;
      const float* hb = Hs + (16 * th + c) * kGP + g;
#pragma unroll
      for (int ks = 0; ks < 16; ++ks)
        a4 = __builtin_amdgcn_mfma_f32_16x16x4f32(ga[4 * ks], hb[4 * ks], a4, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) base[(4 * g + r) * 16 + c] = a4[r];
    }
  }
}

// Backward through one conditioner MLP with output gradient gout[DT]:
// adds d/dc into gc[DC], stages (G, H) and accumulates the weight gradient.
template <int D, int H1, int H2>
__device__ __forceinline__ void net_backward(const float* __restrict__ w, const float* c,
                                             const float* h1, const float* h2,
                                             const float* gout, float* gc, float* Gs, float* Hs,
                                             float* acc, bool valid, int lane) {
  using S = VS<D, H1, H2>;
  constexpr int DT = S::DT, DC = S::DC;
  float G[S::GS], Hv[S::HS];
  float gin[DC];
  if constexpr (H1 == 0) {
    linear_t<DC, D, DT>(w, gout, gin);
#pragma unroll
    for (int j = 0; j < DT; ++j) G[j] = gout[j];
#pragma unroll
    for (int k = 0; k < DC; ++k) Hv[k] = c[k];
  } else if constexpr (H2 == 0) {
    float gh1[H1];
    linear_t<H1, D, DT>(w + Lin<DC, H1>::floats, gout, gh1);
#pragma unroll
    for (int m = 0; m < H1; ++m) gh1[m] = h1[m] > 0.f ? gh1[m] : 0.f;
    linear_t<DC, H1, H1>(w, gh1, gin);
#pragma unroll
    for (int m = 0; m < H1; ++m) G[m] = gh1[m];
#pragma unroll
    for (int j = 0; j < DT; ++j) G[H1 + j] = gout[j];
#pragma unroll
    for (int k = 0; k < DC; ++k) Hv[k] = c[k];
#pragma unroll
    for (int m = 0; m < H1; ++m) Hv[DC + m] = h1[m];
  } else {
    const float* w2 = w + Lin<DC, H1>::floats;
    const float* w3 = w2 + Lin<H1, H2>::floats;
    float gh2[H2], gh1[H1];
    linear_t<H2, D, DT>(w3, gout, gh2);
#pragma unroll
    for (int k = 0; k < H2; ++k) gh2[k] = h2[k] > 0.f ? gh2[k] : 0.f;
    linear_t<H1, H2, H2>(w2, gh2, gh1);
#pragma unroll
    for (int m = 0; m < H1; ++m) gh1[m] = h1[m] > 0.f ? gh1[m] : 0.f;
    linear_t<DC, H1, H1>(w, gh1, gin);
#pragma unroll
    for (int m = 0; m < H1; ++m) G[m] = gh1[m];
#pragma unroll
    for (int k = 0; k < H2; ++k) G[H1 + k] = gh2[k];
#pragma unroll
    for (int j = 0; j < DT; ++j) G[H1 + H2 + j] = gout[j];
#pragma unroll
    for (int k = 0; k < DC; ++k) Hv[k] = c[k];
#pragma unroll
    for (int m = 0; m < H1; ++m) Hv[DC + m] = h1[m];
#pragma unroll
    for (int k = 0; k < H2; ++k) Hv[DC + H1 + k] = h2[k];
  }
  Hv[S::HS - 1] = 1.f;
#pragma unroll
  for (int k = 0; k < DC; ++k) gc[k] += gin[k];
  wave_sync();  // previous accumulate() is done reading the stage
#pragma unroll
  for (int i = 0; i < S::GS; ++i) Gs[i * kGP + lane] = valid ? G[i] : 0.f;
#pragma unroll
  for (int i = 0; i < S::HS; ++i) Hs[i * kGP + lane] = Hv[i];
  wave_sync();
  accumulate<S::TG, S::TH>(acc, Gs, Hs, lane);
}

template <int D, int H1, int H2, bool LOSS>
__global__ __launch_bounds__(kVRows) void k_vjp(
    const float* __restrict__ W, const int32_t* __restrict__ fq,
    const int32_t* __restrict__ iq, const int32_t* __restrict__ lflag,
    const float* __restrict__ x, const int64_t* __restrict__ y, const float* __restrict__ gz,
    const float* __restrict__ gz_all, const float* __restrict__ gld_in, float* __restrict__ dx,
    float* __restrict__ partials, int64_t B, int L, int scale, int shift, int any_perm, int kind,
    float det, float grad_scale, int P, int PS) {
  using S = VS<D, H1, H2>;
  constexpr int DT = S::DT, DC = S::DC;
  constexpr int NF = Net<D, H1, H2>::floats;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x;
  const int nets = scale + shift;
  const int layer_floats = nets * NF;
  float* stash = smem;                                  // [L][DT][64]
  float* Gs = stash + L * DT * kVRows;                  // [16 TG][kGP]
  float* Hs = Gs + 16 * S::TG * kGP;                    // [16 TH][kGP]
  float* acc = Hs + 16 * S::TH * kGP;                   // [L][nets][ACC]
  const int nacc = L * nets * S::ACC;
  for (int i = lane; i < nacc; i += kVRows) acc[i] = 0.f;
  for (int i = lane; i < 16 * (S::TG + S::TH) * kGP; i += kVRows) Gs[i] = 0.f;
  wave_sync();

  float lt0 = 0.f, lt1 = 0.f, lt2 = 0.f;
  const int64_t ntiles = (B + kVRows - 1) / kVRows;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t row = tile * kVRows + lane;
    const bool valid = row < B;
    float v[D];
#pragma unroll
    for (int k = 0; k < D; ++k) v[k] = valid ? x[row * D + k] : 0.f;

    // ---- forward sweep (stash the transformed inputs) --------------------
    float ld = 0.f;
    auto fwd = [&](auto O_, int l) __attribute__((always_inline)) {
      constexpr bool O = decltype(O_)::value;
#pragma unroll
      for (int j = 0; j < DT; ++j) stash[(l * DT + j) * kVRows + lane] = v[R<D, O>(j)];
      const bool pm = any_perm && (lflag[l] & kFlagPerm);
      step<D, H1, H2, false, false, O, true, false>(v, ld, W + (int64_t)l * layer_floats, scale,
                                                    shift, NF, pm, fq + l * D);
    };
    int l = 0;
    for (; l + 1 < L; l += 2) {
      fwd(std::false_type{}, l);
      fwd(std::true_type{}, l + 1);
    }
    const bool oddL = l < L;
    if (oddL) fwd(std::false_type{}, l);

    // ---- upstream gradient at z_L (orientation OL = L & 1) ---------------
    float g[D];
    float gld = 0.f;
    auto seed = [&](auto O_) __attribute__((always_inline)) {
      constexpr bool O = decltype(O_)::value;
      if constexpr (LOSS) {
        float z[D];
#pragma unroll
        for (int j = 0; j < D; ++j) z[j] = v[R<D, O>(j)];
        float m = z[0];
#pragma unroll
        for (int j = 1; j < D; ++j) m = fmaxf(m, z[j]);
        float se = 0.f;
#pragma unroll
        for (int j = 0; j < D; ++j) se += expf(z[j] - m);
        const float lse = m + logf(se);
        // a label outside [0, D) poisons this row's loss and gradient with NaN
        // (the reference's probs.gather raises on it)
        const int64_t yr = valid ? y[row] : 0;
        const bool yok = yr >= 0 && yr < D;
        const int yy = yok ? (int)yr : 0;
        float zy = z[0];
#pragma unroll
        for (int j = 1; j < D; ++j) zy = (j == yy) ? opaque(z[j]) : zy;
        const float lpy = zy - lse;
        float coef, ce_term, loss_row;
        if (kind == CNF_LOSS_CAL) {  // -(log(softmax(z)[y] + 1e-7) + ld)
          const float py = expf(lpy);
          ce_term = -logf(py + kEps);
          loss_row = ce_term - ld;
          coef = py / (py + kEps);
          gld = -grad_scale;
        } else {                     // CE(z, y) - det * ld
          ce_term = -lpy;
          loss_row = ce_term - det * ld;
          coef = 1.f;
          gld = -det * grad_scale;
        }
        if (!yok) ce_term = loss_row = coef = __builtin_nanf("");
#pragma unroll
        for (int j = 0; j < D; ++j) {
          const float p = expf(z[j] - lse);
          g[R<D, O>(j)] = grad_scale * coef * (p - (j == yy ? 1.f : 0.f));
        }
        if (valid) {
          lt0 += loss_row;
          lt1 += ce_term;
          lt2 += ld;
        } else {
          gld = 0.f;
#pragma unroll
          for (int j = 0; j < D; ++j) g[j] = 0.f;
        }
      } else {
#pragma unroll
        for (int j = 0; j < D; ++j) g[R<D, O>(j)] = (gz && valid) ? gz[row * D + j] : 0.f;
        gld = (gld_in && valid) ? gld_in[row] : 0.f;
      }
    };
    if (oddL) seed(std::true_type{});
    else seed(std::false_type{});

    // ---- backward sweep ---------------------------------------------------
    auto bwd = [&](auto Oc_, int l) __attribute__((always_inline)) {
      constexpr bool Oc = decltype(Oc_)::value;  // orientation of z_l
      constexpr bool Oi = !Oc;
      if (gz_all && valid) {
        const float* ga = gz_all + ((int64_t)l * B + row) * D;
#pragma unroll
        for (int j = 0; j < D; ++j) g[R<D, Oc>(j)] += ga[j];
      }
      // undo z[:, perm].flip(1): z_pre[i] = z_out[iq[i]]
      if (any_perm && (lflag[l] & kFlagPerm)) {
        permute<D, Oc>(v, iq + l * D);
        permute<D, Oc>(g, iq + l * D);
      }
      float c[DC], xT[DT];
#pragma unroll
      for (int k = 0; k < DC; ++k) c[k] = v[R<D, Oi>(DT + k)];
#pragma unroll
      for (int j = 0; j < DT; ++j) xT[j] = stash[(l * DT + j) * kVRows + lane];
      const float* wl = W + (int64_t)l * layer_floats;
      float gc[DC];
#pragma unroll
      for (int k = 0; k < DC; ++k) gc[k] = 0.f;
      float gxT[DT];
      float* accl = acc + (int64_t)l * nets * S::ACC;
      constexpr int H1s = H1 > 0 ? H1 : 1, H2s = H2 > 0 ? H2 : 1;
      if (scale) {
        float h1[H1s], h2[H2s], s[DT];
        mlp_keep<D, H1, H2>(wl, c, h1, h2, s);
        float gs[DT];
#pragma unroll
        for (int j = 0; j < DT; ++j) {
          const float gzj = g[R<D, Oi>(j)];
          const float e = __expf(s[j]);
          gs[j] = gzj * xT[j] * e + gld;   // z = x e^s + t ; ld += s
          gxT[j] = gzj * e;
        }
        net_backward<D, H1, H2>(wl, c, h1, h2, gs, gc, Gs, Hs, accl, valid, lane);
        accl += S::ACC;
        wl += NF;
      } else {
#pragma unroll
        for (int j = 0; j < DT; ++j) gxT[j] = g[R<D, Oi>(j)];
      }
      if (shift) {
        float h1[H1s], h2[H2s], t[DT];
        mlp_keep<D, H1, H2>(wl, c, h1, h2, t);  // only the activations are needed
        float gt[DT];
#pragma unroll
        for (int j = 0; j < DT; ++j) gt[j] = g[R<D, Oi>(j)];
        net_backward<D, H1, H2>(wl, c, h1, h2, gt, gc, Gs, Hs, accl, valid, lane);
      }
#pragma unroll
      for (int j = 0; j < DT; ++j) {
        v[R<D, Oi>(j)] = xT[j];
        g[R<D, Oi>(j)] = gxT[j];
      }
#pragma unroll
      for (int k = 0; k < DC; ++k) g[R<D, Oi>(DT + k)] += gc[k];
    };
    int lb = L - 1;
    if ((lb & 1) == 0) {  // layer L-1 even: its output orientation is 1
      bwd(std::true_type{}, lb);
      --lb;
    }
    for (; lb >= 1; lb -= 2) {
      bwd(std::false_type{}, lb);
      bwd(std::true_type{}, lb - 1);
    }
    if (dx && valid) {
#pragma unroll
      for (int j = 0; j < D; ++j) dx[row * D + j] = g[j];
    }
  }

  // ---- this block's partial sums, natural (state_dict) parameter order ----
  wave_sync();
  float* out = partials + (int64_t)blockIdx.x * PS;
  const int nfn = S::NFN;
  for (int p = lane; p < P; p += kVRows) {
    const int l = p / (nets * nfn);
    int r = p - l * nets * nfn;
    const int n = r / nfn;
    r -= n * nfn;
    // walk the net's Linear layers: units [D, H1?, H2?, D]
    int nu = 0;
    int u[4];
    u[nu++] = D;
    if (H1) u[nu++] = H1;
    if (H2) u[nu++] = H2;
    u[nu++] = D;
    int gofs = 0, hofs = 0, gi = -1, hi = -1;
    for (int i = 0; i < nu - 1; ++i) {
      const int nin = u[i], nout = u[i + 1];
      const bool first = i == 0, last = i == nu - 2;
      const int nout_eff = last ? DT : nout;
      const int nin_eff = first ? DC : nin;
      if (r < nout * nin) {
        const int o = r / nin, col = r - (r / nin) * nin;
        const int kk = first ? col - DT : col;
        if (o < nout_eff && kk >= 0 && kk < nin_eff) {
          gi = gofs + o;
          hi = hofs + kk;
        }
        break;
      }
      r -= nout * nin;
      if (r < nout) {
        if (r < nout_eff) {
          gi = gofs + r;
          hi = S::HS - 1;
        }
        break;
      }
      r -= nout;
      gofs += nout_eff;
      hofs += nin_eff;
    }
    float val = 0.f;
    if (gi >= 0) {
      const int tg = gi >> 4, ii = gi & 15, th = hi >> 4, jj = hi & 15;
      val = acc[((int64_t)l * nets + n) * S::ACC + (tg * S::TH + th) * 256 + ii * 16 + jj];
    }
    out[p] = val;
  }
  if (LOSS) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      lt0 += __shfl_xor(lt0, off);
      lt1 += __shfl_xor(lt1, off);
      lt2 += __shfl_xor(lt2, off);
    }
    if (lane == 0) {
      out[P] = lt0;
      out[P + 1] = lt1;
      out[P + 2] = lt2;
    }
  }
}

// Fixed-order reductions of the per-block partials partials[b][0..NE) (row
// stride PS) -- deterministic: every entry is always summed in the same tree.
//
// Many entries (weight gradients): a block owns 64 consecutive entries and
// its 4 waves split the blocks b = g, g+4, ... (coalesced 256-B rows); the 4
// group sums are then added in group order.
// Column sums of per-block partial records: block (x, y) adds rows
// [y*R, min(nblk, (y+1)*R)) of columns [64x, 64x + 64) -- four row groups of
// 64 lanes, four loads in flight each -- and writes the sums to out + y*ostride
// (ostride = R*PS: in place over the chunk's first row, which only this block
// reads).  grid.y = 1 gives the final sums.  Fixed grouping: deterministic.
__global__ __launch_bounds__(256) void k_reduce_cols(const float* __restrict__ partials, int nblk,
                                                     int PS, int NE, float* __restrict__ out,
                                                     int R, int64_t ostride) {
  __shared__ float red[256];
  const int e = blockIdx.x * 64 + (threadIdx.x & 63), g = threadIdx.x >> 6;
  const int r0 = (int)blockIdx.y * R, n = min(R, nblk - r0);
  const float* base = partials + (int64_t)r0 * PS;
  float s = 0.f;
  if (e < NE) {
    int b = g;
    for (; b + 12 < n; b += 16) {
      const float a0 = base[(int64_t)b * PS + e], a1 = base[(int64_t)(b + 4) * PS + e];
      const float a2 = base[(int64_t)(b + 8) * PS + e];
      const float a3 = base[(int64_t)(b + 12) * PS + e];
      s += a0;
      s += a1;
      s += a2;
      s += a3;
    }
    for (; b < n; b += 4) s += base[(int64_t)b * PS + e];
  }
  red[threadIdx.x] = s;
  __syncthreads();
  if (g == 0 && e < NE)
    out[(int64_t)blockIdx.y * ostride + e] =
        ((red[threadIdx.x] + red[threadIdx.x + 64]) + red[threadIdx.x + 128]) +
        red[threadIdx.x + 192];
}

// The 3 loss sums: ONE wave.  Lane l adds blocks l, l+64, ... in order (eight
// blocks' loads in flight per batch), then a fixed xor-butterfly over the 64
// lanes -- no LDS, no barrier; deterministic for a given nblk.  This launch
// sits on the critical path after the main pass, so its latency is the cost.
__global__ __launch_bounds__(64) void k_reduce_rows(const float* __restrict__ partials, int nblk,
                                                    int PS, int E0, int NE,
                                                    float* __restrict__ out) {
  const int l = threadIdx.x;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f;
  for (int b0 = l; b0 < nblk; b0 += 8 * 64) {
    float v[8][3];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int b = b0 + k * 64;
      const float* p = partials + (int64_t)b * PS + E0;
      v[k][0] = b < nblk ? p[0] : 0.f;
      v[k][1] = b < nblk && NE > 1 ? p[1] : 0.f;
      v[k][2] = b < nblk && NE > 2 ? p[2] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      s0 += v[k][0];
      s1 += v[k][1];
      s2 += v[k][2];
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    s0 += __shfl_xor(s0, off);
    s1 += __shfl_xor(s1, off);
    s2 += __shfl_xor(s2, off);
  }
  if (l == 0) {
    out[0] = s0;
    if (NE > 1) out[1] = s1;
    if (NE > 2) out[2] = s2;
  }
}

// Loss-term sums of 16-B partial records ([t0, t1, t2, pad] per block, the
// forward-loss kernels' layout): four waves, one float4 per record, up to
// eight records per lane in flight before the first add, so a 2,048-block grid
// is one round of load latency instead of four.  Fixed order throughout
// (lane-strided sums, xor butterfly, waves in index order): deterministic.
constexpr int kRR = 256;
__global__ __launch_bounds__(kRR) void k_reduce_rows4(const float4* __restrict__ partials,
                                                      int nblk, float* __restrict__ out) {
  __shared__ float red[kRR / 64][3];
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
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    s0 += __shfl_xor(s0, off);
    s1 += __shfl_xor(s1, off);
    s2 += __shfl_xor(s2, off);
  }
  if ((t & 63) == 0) {
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

// ===========================================================================
// k_vjp2: reverse mode on packed row pairs (two rows per lane, v_pk_fma_f32)
// with the weights as SGPR operands (the plain packed-SGPR region), for the
// narrow shapes whose conditioner gradient stacks fit one 16x16 MFMA tile
// (GS = H1 + H2 + D/2 <= 16, HS = D - D/2 + H1 + H2 + 1 <= 16) and L <= 8.
//
// One wave per block walks tiles of 128 rows (grid-strided):
//   forward   the L layers, each layer's transformed-half input x_T stashed
//             in the workspace (HBM scratch, written and re-read by the same
//             wave within the tile: L2-resident in practice);
//   seed      the loss gradient (or gz / gld / gz_all of a generic VJP);
//   backward  per layer, last to first: undo flip / perm (renaming), recompute
//             both conditioners on the conditioning half, take the layer's
//             input x_T from the stash (recovering it as (z_T - t) exp(-s)
//             loses the reference's precision once |s| is large), back-
//             propagate through the affine update
//             and both MLPs (transposed products on SGPR weights);
//   dW        each net's G = [g_a1, g_a2, g_out] and H = [c, h1, h2, 1] go
//             through a 16 KB LDS stage 64 rows at a time and are folded into a
//             16x16 accumulator by v_mfma_f32_16x16x4f32 with the rows as K;
//             the accumulators of all (layer, net) live in registers for the
//             wave's whole run and are written once, as this wave's partial.
// Partials are summed in wave order by k_reduce_cols (deterministic).
// ===========================================================================
template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

constexpr int kV2TR = 128;   // rows per wave tile (lane l: rows 2l, 2l+1)
constexpr int kV2LMax = 8;   // layers the register accumulators hold
constexpr int kV2SS = 68;    // stage row stride in floats (64 rows + pad, 16-B aligned)

struct VArgs2 {
  const float* x;
  const int64_t* y;
  const float* gz;
  const float* gz_all;
  const float* gld;
  float* dx;
  float* partials;
  float* stash;  // [L][B][D/2] transformed-half layer inputs
  int64_t B;
  int L, kind;
  float det, grad_scale;
  int P, PS;
};

// widx: W[o][k] in the packed row layout [w_o0, b_o, w_o1 .. ] at stride S
template <int S>
__device__ __forceinline__ constexpr int widx(int o, int k) { return o * S + (k == 0 ? 0 : 1 + k); }

// y[o] = b[o] + sum_k W[o][k] x[k], o < NOUT (plain weights; input-major chains)
template <int NIN, int NOUT, int S, bool RELU, int NC>
__device__ __forceinline__ void vlin(const SW<NC>& w, const f2* x, f2* y) {
  f2 a[NOUT];
#pragma unroll
  for (int o = 0; o < NOUT; ++o) a[o] = fma_wb(w.pair(o * S), x[0]);
#pragma unroll
  for (int k = 1; k < NIN; ++k)
#pragma unroll
    for (int o = 0; o < NOUT; ++o) a[o] = fmaT(w[widx<S>(o, k)], x[k], a[o]);
#pragma unroll
  for (int o = 0; o < NOUT; ++o) y[o] = RELU ? maxT(a[o], splat(0.f, f2{})) : a[o];
}

// gin[k] = sum_o W[o][k] gout[o], k < NIN, o < NOUT
template <int NIN, int NOUT, int S, int NC>
__device__ __forceinline__ void vlin_t(const SW<NC>& w, const f2* gout, f2* gin) {
#pragma unroll
  for (int k = 0; k < NIN; ++k) gin[k] = gout[0] * splat(w[widx<S>(0, k)], f2{});
#pragma unroll
  for (int o = 1; o < NOUT; ++o)
#pragma unroll
    for (int k = 0; k < NIN; ++k) gin[k] = fmaT(w[widx<S>(o, k)], gout[o], gin[k]);
}

template <int NC>
__device__ __forceinline__ void sload_now(SW<NC>& w, const float* p) {
  sissue(w, p);
  sready();
}

// One net's activations on the conditioning half c (plain weights): h1, h2, out.
template <class S, int NC>
__device__ __forceinline__ void vnet_fwd(const float* wn, const f2* c, f2* h1, f2* h2, f2* out) {
  SW<NC> w;
  if constexpr (S::NL == 1) {
    sload_now(w, wn);
    vlin<S::nin(0), S::nout(0), S::stride(0), false>(w, c, out);
  } else if constexpr (S::NL == 2) {
    sload_now(w, wn);
    vlin<S::nin(0), S::nout(0), S::stride(0), true>(w, c, h1);
    sload_now(w, wn + S::off(1));
    vlin<S::nin(1), S::nout(1), S::stride(1), false>(w, h1, out);
  } else {
    sload_now(w, wn);
    vlin<S::nin(0), S::nout(0), S::stride(0), true>(w, c, h1);
    sload_now(w, wn + S::off(1));
    vlin<S::nin(1), S::nout(1), S::stride(1), true>(w, h1, h2);
    sload_now(w, wn + S::off(2));
    vlin<S::nin(2), S::nout(2), S::stride(2), false>(w, h2, out);
  }
}

// Back-propagate one net: gout (d/d out) -> adds d/dc into gc and leaves the
// gradient stack G = [g_a1, g_a2, gout] (pre-activation gradients).
template <class S, int NC>
__device__ __forceinline__ void vnet_bwd(const float* wn, const f2* h1, const f2* h2,
                                         const f2* gout, f2* gc, f2* G) {
  constexpr int H1 = S::NL >= 2 ? S::nout(0) : 0, H2 = S::NL == 3 ? S::nout(1) : 0;
  constexpr int DT = S::DT, DC = S::DC;
  SW<NC> w;
  f2 gin[DC];
  const f2 zero = splat(0.f, f2{});
  if constexpr (S::NL == 1) {
    sload_now(w, wn);
    vlin_t<DC, DT, S::stride(0)>(w, gout, gin);
  } else if constexpr (S::NL == 2) {
    f2 g1[H1];
    sload_now(w, wn + S::off(1));
    vlin_t<H1, DT, S::stride(1)>(w, gout, g1);
#pragma unroll
    for (int m = 0; m < H1; ++m) {
      const f2 h = h1[m];
      g1[m] = f2{h.x > 0.f ? g1[m].x : 0.f, h.y > 0.f ? g1[m].y : 0.f};
      G[m] = g1[m];
    }
    sload_now(w, wn);
    vlin_t<DC, H1, S::stride(0)>(w, g1, gin);
  } else {
    f2 g2[H2], g1[H1];
    sload_now(w, wn + S::off(2));
    vlin_t<H2, DT, S::stride(2)>(w, gout, g2);
#pragma unroll
    for (int m = 0; m < H2; ++m) {
      const f2 h = h2[m];
      g2[m] = f2{h.x > 0.f ? g2[m].x : 0.f, h.y > 0.f ? g2[m].y : 0.f};
      G[H1 + m] = g2[m];
    }
    sload_now(w, wn + S::off(1));
    vlin_t<H1, H2, S::stride(1)>(w, g2, g1);
#pragma unroll
    for (int m = 0; m < H1; ++m) {
      const f2 h = h1[m];
      g1[m] = f2{h.x > 0.f ? g1[m].x : 0.f, h.y > 0.f ? g1[m].y : 0.f};
      G[m] = g1[m];
    }
    sload_now(w, wn);
    vlin_t<DC, H1, S::stride(0)>(w, g1, gin);
  }
#pragma unroll
  for (int j = 0; j < DT; ++j) G[H1 + H2 + j] = gout[j];
#pragma unroll
  for (int k = 0; k < DC; ++k) gc[k] += gin[k];
  (void)zero;
}

// Fold G^T H of this tile's 128 rows (GS x HS <= 16 x 16) into acc: the stage
// holds 64 rows at a time ([feature][row], G features 0..15 then H 16..31);
// lane l feeds MFMA step ks with feature l%16 of row (l/16)*16 + ks, so its
// operands for all 16 steps are 16 contiguous floats (4 ds_read_b128).
template <int GS, int HS>
__device__ __forceinline__ floatx4 wgrad_tile(float* st, const f2* G, const f2* H, int lane,
                                              floatx4 acc) {
#pragma unroll
  for (int ch = 0; ch < 2; ++ch) {
    wave_sync();  // the previous reads of the stage are done
#pragma unroll
    for (int f = 0; f < GS; ++f) st[f * kV2SS + lane] = ch ? G[f].y : G[f].x;
#pragma unroll
    for (int f = 0; f < HS; ++f) st[(16 + f) * kV2SS + lane] = ch ? H[f].y : H[f].x;
    wave_sync();
    const float4* ga = reinterpret_cast<const float4*>(st + (lane & 15) * kV2SS + (lane >> 4) * 16);
    const float4* hb =
        reinterpret_cast<const float4*>(st + (16 + (lane & 15)) * kV2SS + (lane >> 4) * 16);
    float4 A[4], Bv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      A[q] = ga[q];
      Bv[q] = hb[q];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A[q].x, Bv[q].x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A[q].y, Bv[q].y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A[q].z, Bv[q].z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A[q].w, Bv[q].w, acc, 0, 0, 0);
    }
  }
  return acc;
}

// parameter p (state_dict order of one layer) -> (G row i, H column j) of its
// gradient in the (layer, net) tile, or -1 when the gradient is zero by the mask
// (the transformed-half inputs of the first Linear, the conditioning-half
// outputs of the last).  Returns the net index through *net.
template <int D, int H1, int H2, int NETS>
__device__ __forceinline__ int param_cell(int r, int* net) {
  using S = SP<D, H1, H2>;
  constexpr int DT = S::DT, DC = S::DC, NL = S::NL;
  constexpr int U[4] = {D, H1 ? H1 : D, H2 ? H2 : D, D};
  constexpr int NFN = H1 == 0 ? D * D + D : (H2 == 0 ? H1 * D + H1 + D * H1 + D
                                                      : H1 * D + H1 + H2 * H1 + H2 + D * H2 + D);
  constexpr int HS = DC + H1 + H2 + 1;
  *net = r / NFN;
  r -= *net * NFN;
  int gofs = 0, hofs = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int nin = U[i], nout = i == NL - 1 ? D : U[i + 1];
    const bool first = i == 0, last = i == NL - 1;
    const int nout_eff = last ? DT : nout, nin_eff = first ? DC : nin;
    if (r < nout * nin) {
      const int o = r / nin, col = r - o * nin;
      const int kk = first ? col - DT : col;
      return (o < nout_eff && kk >= 0 && kk < nin_eff) ? (gofs + o) * 16 + hofs + kk : -1;
    }
    r -= nout * nin;
    if (r < nout) return r < nout_eff ? (gofs + r) * 16 + HS - 1 : -1;
    r -= nout;
    gofs += nout_eff;
    hofs += nin_eff;
  }
  return -1;
}

// accumulator cell (G row i, H column j) -> offset of its parameter in the
// net's state_dict block, or -1 (a cell of the dense tile with no parameter)
template <int D, int H1, int H2>
__device__ __forceinline__ int cell_param(int i, int j) {
  using S = SP<D, H1, H2>;
  constexpr int DT = S::DT, DC = S::DC, NL = S::NL;
  constexpr int U[4] = {D, H1 ? H1 : D, H2 ? H2 : D, D};
  constexpr int HS = DC + H1 + H2 + 1;
  int gofs = 0, hofs = 0, woff = 0;
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const int nin = U[k], nout = k == NL - 1 ? D : U[k + 1];
    const bool first = k == 0, last = k == NL - 1;
    const int nout_eff = last ? DT : nout, nin_eff = first ? DC : nin, in_off = first ? DT : 0;
    if (i >= gofs && i < gofs + nout_eff) {
      const int o = i - gofs;
      if (j == HS - 1) return woff + nout * nin + o;
      if (j >= hofs && j < hofs + nin_eff) return woff + o * nin + in_off + (j - hofs);
      return -1;
    }
    woff += nout * nin + nout;
    gofs += nout_eff;
    hofs += nin_eff;
  }
  return -1;
}

template <int D, int H1, int H2, int NETS, bool LOSS, bool PERM>
__global__ __launch_bounds__(64, 2) void k_vjp2(const float* __restrict__ W,
                                                const int32_t* __restrict__ fq,
                                                const int32_t* __restrict__ iq,
                                                const int32_t* __restrict__ lflag, VArgs2 a) {
  using S = SP<D, H1, H2>;
  constexpr int DT = S::DT, DC = S::DC, NC = S::NC;
  constexpr int LF = NETS * S::NF;
  constexpr int GS = H1 + H2 + DT, HS = DC + H1 + H2 + 1;
  static_assert(GS <= 16 && HS <= 16, "gradient stacks must fit one 16x16 MFMA tile");
  constexpr int TF = kV2TR * D;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* tile = smem;        // [TF] input rows
  float* st = smem + TF;     // [32][kV2SS] G / H stage
  const int lane = threadIdx.x;
  const int64_t B = a.B;
  const int L = a.L;
  const int ntiles = (int)((B + kV2TR - 1) / kV2TR);
  const f2 zero = splat(0.f, f2{});
  constexpr float kLN2 = 0.69314718055994531f, kL2E = 1.4426950408889634f;
  floatx4 acc[kV2LMax][NETS];
#pragma unroll
  for (int l = 0; l < kV2LMax; ++l)
#pragma unroll
    for (int n = 0; n < NETS; ++n) acc[l][n] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int i = lane; i < 32 * kV2SS; i += 64) st[i] = 0.f;
  float lt0 = 0.f, lt1 = 0.f, lt2 = 0.f;

  for (int tix = blockIdx.x; tix < ntiles; tix += gridDim.x) {
    const int64_t row0 = (int64_t)tix * kV2TR;
    const int64_t r = row0 + 2 * lane;
    const int nr = r >= B ? 0 : (r + 1 >= B ? 1 : 2);
    // ---- rows in: one tile through LDS (full tiles: 16-B loads) ----
    f2 v[D];
    if (row0 + kV2TR <= B) {
      wave_sync();
      const float4* s4 = reinterpret_cast<const float4*>(a.x + row0 * D);
      float4* d4 = reinterpret_cast<float4*>(tile);
      for (int i = lane; i < TF / 4; i += 64) d4[i] = s4[i];
      wave_sync();
      f2 vv[1][D];
      read_pairs<D, 1>(tile, lane, vv);
#pragma unroll
      for (int k = 0; k < D; ++k) v[k] = vv[0][k];
    } else {
#pragma unroll
      for (int k = 0; k < D; ++k)
        v[k] = f2{nr > 0 ? a.x[r * D + k] : 0.f, nr > 1 ? a.x[(r + 1) * D + k] : 0.f};
    }
    uint32_t lab = 0;
    if constexpr (LOSS) lab = load_labels<D, 1>(a.y + r, nr, false);

    // ---- forward sweep (plain weights, nothing stashed) ----
    f2 ld = zero;
    auto fwd = [&](auto O_, int l) __attribute__((always_inline)) {
      constexpr bool O = decltype(O_)::value;
      const float* wl = W + (int64_t)l * LF;
      f2 c[DC];
#pragma unroll
      for (int k = 0; k < DC; ++k) c[k] = v[R<D, O>(DT + k)];
      f2 h1[H1 ? H1 : 1], h2[H2 ? H2 : 1], t[DT], sv[DT];
      {  // x_T of this layer, rows r, r+1: 2*DT contiguous floats
        float* sp = a.stash + ((int64_t)l * B + r) * DT;
#pragma unroll
        for (int j = 0; j < DT; ++j) {
          if (nr > 0) sp[j] = v[R<D, O>(j)].x;
          if (nr > 1) sp[DT + j] = v[R<D, O>(j)].y;
        }
      }
      vnet_fwd<S, NC>(wl + (NETS == 2 ? S::NF : 0), c, h1, h2, t);
      if constexpr (NETS == 2) vnet_fwd<S, NC>(wl, c, h1, h2, sv);
#pragma unroll
      for (int j = 0; j < DT; ++j) {
        f2& x = v[R<D, O>(j)];
        if constexpr (NETS == 2) {
          x = fmaV(x, exp2T(sv[j] * splat(kL2E, f2{})), t[j]);
          ld += sv[j];
        } else {
          x += t[j];
        }
      }
      if constexpr (PERM) {
        if (lflag[l] & kFlagPerm) permute<D, O>(v, fq + l * D);
      }
    };
    int l = 0;
    for (; l + 1 < L; l += 2) {
      fwd(std::false_type{}, l);
      fwd(std::true_type{}, l + 1);
    }
    const bool oddL = l < L;
    if (oddL) fwd(std::false_type{}, l);

    // ---- upstream gradient at z_L (orientation L & 1) ----
    f2 g[D];
    f2 gld = zero;
    auto seed = [&](auto O_) __attribute__((always_inline)) {
      constexpr bool O = decltype(O_)::value;
      if constexpr (LOSS) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          float z[D];
#pragma unroll
          for (int j = 0; j < D; ++j) z[j] = v[R<D, O>(j)][q];
          float m = z[0];
#pragma unroll
          for (int j = 1; j < D; ++j) m = fmaxf(m, z[j]);
          float se = 0.f;
#pragma unroll
          for (int j = 0; j < D; ++j) se += __builtin_amdgcn_exp2f((z[j] - m) * kL2E);
          const float lse = m + __builtin_amdgcn_logf(se) * kLN2;
          const uint32_t b = (lab >> (8 * q)) & 0xffu;
          const bool ok = b != 0xffu, valid = q < nr;
          const int yy = ok ? (int)b : 0;
          uint32_t zb[D];
#pragma unroll
          for (int j = 0; j < D; ++j) zb[j] = __float_as_uint(z[j]);
          const float lpy = __uint_as_float(sel_tree<D>(zb, yy, 0)) - lse;
          const float ldq = NETS == 2 ? ld[q] : 0.f;  // plain weights: ld = sum(s)
          float coef, ce_term, loss_row, gl;
          if (a.kind == CNF_LOSS_CAL) {  // -(log(softmax(z)[y] + 1e-7) + ld)
            const float py = __builtin_amdgcn_exp2f(lpy * kL2E);
            ce_term = -__builtin_amdgcn_logf(py + kEps) * kLN2;
            loss_row = ce_term - ldq;
            coef = py / (py + kEps);
            gl = -a.grad_scale;
          } else {                       // CE(z, y) - det * ld
            ce_term = -lpy;
            loss_row = ce_term - a.det * ldq;
            coef = 1.f;
            gl = -a.det * a.grad_scale;
          }
          if (!ok) ce_term = loss_row = coef = __builtin_nanf("");
          if (!valid) coef = gl = 0.f;
#pragma unroll
          for (int j = 0; j < D; ++j) {
            const float pj = __builtin_amdgcn_exp2f((z[j] - lse) * kL2E);
            g[R<D, O>(j)][q] = a.grad_scale * coef * (pj - (j == yy ? 1.f : 0.f));
          }
          gld[q] = gl;
          if (valid) {
            lt0 += loss_row;
            lt1 += ce_term;
            lt2 += ldq;
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < D; ++j)
          g[R<D, O>(j)] = f2{a.gz && nr > 0 ? a.gz[r * D + j] : 0.f,
                              a.gz && nr > 1 ? a.gz[(r + 1) * D + j] : 0.f};
        gld = f2{a.gld && nr > 0 ? a.gld[r] : 0.f, a.gld && nr > 1 ? a.gld[r + 1] : 0.f};
      }
    };
    if (oddL) seed(std::true_type{});
    else seed(std::false_type{});

    // ---- backward sweep ----
    // layer index compile-time (static_for below): the per-layer gradient
    // accumulators acc[l][net] stay in registers (a runtime-indexed select
    // over them was lowered to scratch)
    auto bwd = [&](auto LI) __attribute__((always_inline)) {
      constexpr int l = decltype(LI)::value;
      constexpr bool Oc = ((l + 1) & 1) != 0;  // orientation of z_l
      constexpr bool Oi = !Oc;
      if (a.gz_all) {
#pragma unroll
        for (int j = 0; j < D; ++j)
          g[R<D, Oc>(j)] += f2{nr > 0 ? a.gz_all[((int64_t)l * B + r) * D + j] : 0.f,
                               nr > 1 ? a.gz_all[((int64_t)l * B + r + 1) * D + j] : 0.f};
      }
      if constexpr (PERM) {
        if (lflag[l] & kFlagPerm) {  // undo z[:, perm].flip(1): z_pre[i] = z_out[iq[i]]
          permute<D, Oc>(v, iq + l * D);
          permute<D, Oc>(g, iq + l * D);
        }
      }
      const float* wl = W + (int64_t)l * LF;
      f2 c[DC], gT[DT], gc[DC];
#pragma unroll
      for (int k = 0; k < DC; ++k) {
        c[k] = v[R<D, Oi>(DT + k)];
        gc[k] = zero;
      }
#pragma unroll
      for (int j = 0; j < DT; ++j) gT[j] = g[R<D, Oi>(j)];
      f2 xT[DT];
      {
        const float* sp = a.stash + ((int64_t)l * B + r) * DT;
#pragma unroll
        for (int j = 0; j < DT; ++j) xT[j] = f2{nr > 0 ? sp[j] : 0.f, nr > 1 ? sp[DT + j] : 0.f};
      }
      f2 th1[H1 ? H1 : 1], th2[H2 ? H2 : 1], t[DT];
      vnet_fwd<S, NC>(wl + (NETS == 2 ? S::NF : 0), c, th1, th2, t);
      f2 H[HS];
#pragma unroll
      for (int k = 0; k < DC; ++k) H[k] = c[k];
      H[HS - 1] = splat(1.f, f2{});
      // invalid (padding) rows contribute nothing to the weight gradients
      const f2 keep = f2{nr > 0 ? 1.f : 0.f, nr > 1 ? 1.f : 0.f};
      if constexpr (NETS == 2) {
        f2 sh1[H1 ? H1 : 1], sh2[H2 ? H2 : 1], sv[DT];
        vnet_fwd<S, NC>(wl, c, sh1, sh2, sv);
        f2 gs[DT];
#pragma unroll
        for (int j = 0; j < DT; ++j) {
          const f2 e = exp2T(sv[j] * splat(kL2E, f2{}));
          gs[j] = fmaV(gT[j] * xT[j], e, gld);  // z_T = x_T e^s + t, ld += s
          gT[j] = gT[j] * e;
        }
        f2 G[GS];
        vnet_bwd<S, NC>(wl, sh1, sh2, gs, gc, G);
#pragma unroll
        for (int f = 0; f < GS; ++f) G[f] *= keep;
#pragma unroll
        for (int m = 0; m < H1; ++m) H[DC + m] = sh1[m];
#pragma unroll
        for (int m = 0; m < H2; ++m) H[DC + H1 + m] = sh2[m];
        acc[l][0] = wgrad_tile<GS, HS>(st, G, H, lane, acc[l][0]);
      }
      {  // t-net: d/dt = g_T (before the e^s scaling of the s-net branch)
        f2 G[GS];
        f2 gt[DT];
#pragma unroll
        for (int j = 0; j < DT; ++j) gt[j] = g[R<D, Oi>(j)];
        vnet_bwd<S, NC>(wl + (NETS == 2 ? S::NF : 0), th1, th2, gt, gc, G);
#pragma unroll
        for (int f = 0; f < GS; ++f) G[f] *= keep;
#pragma unroll
        for (int m = 0; m < H1; ++m) H[DC + m] = th1[m];
#pragma unroll
        for (int m = 0; m < H2; ++m) H[DC + H1 + m] = th2[m];
        acc[l][NETS - 1] = wgrad_tile<GS, HS>(st, G, H, lane, acc[l][NETS - 1]);
      }
#pragma unroll
      for (int j = 0; j < DT; ++j) {
        v[R<D, Oi>(j)] = xT[j];
        g[R<D, Oi>(j)] = gT[j];
      }
#pragma unroll
      for (int k = 0; k < DC; ++k) g[R<D, Oi>(DT + k)] += gc[k];
    };
    static_for<0, kV2LMax>([&](auto I) __attribute__((always_inline)) {
      constexpr int l = kV2LMax - 1 - decltype(I)::value;
      if (l < L) bwd(std::integral_constant<int, l>{});
    });
    if (a.dx) {
#pragma unroll
      for (int j = 0; j < D; ++j) {
        if (nr > 0) a.dx[r * D + j] = g[j].x;
        if (nr > 1) a.dx[(r + 1) * D + j] = g[j].y;
      }
    }
  }

  // ---- this wave's partial: parameter gradients (state_dict order) + loss sums ----
  float* out = a.partials + (int64_t)blockIdx.x * a.PS;
  const int P = a.P;
  constexpr int NFN = H1 == 0 ? D * D + D : (H2 == 0 ? H1 * D + H1 + D * H1 + D
                                                      : H1 * D + H1 + H2 * H1 + H2 + D * H2 + D);
  // zeros where the mask makes the gradient vanish
  for (int p = lane; p < P; p += 64) {
    int n;
    const int l = p / (NETS * NFN);
    if (param_cell<D, H1, H2, NETS>(p - l * NETS * NFN, &n) < 0) out[p] = 0.f;
  }
  // the lane's accumulator cells: C[i = 4 (lane/16) + e][j = lane % 16]
  const int j = lane & 15, i0 = 4 * (lane >> 4);
  static_for<0, kV2LMax>([&](auto I) __attribute__((always_inline)) {
    constexpr int l = decltype(I)::value;
    if (l >= L) return;
#pragma unroll
    for (int n = 0; n < NETS; ++n) {
      const floatx4 c4 = acc[l][n];
      // net n's parameters follow the layer's state_dict order: s-net first
      const int base = l * NETS * NFN + n * NFN;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int q = cell_param<D, H1, H2>(i0 + e, j);
        if (q >= 0) out[base + q] = c4[e];
      }
    }
  });
  if constexpr (LOSS) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      lt0 += __shfl_xor(lt0, off);
      lt1 += __shfl_xor(lt1, off);
      lt2 += __shfl_xor(lt2, off);
    }
    if (lane == 0) {
      out[P] = lt0;
      out[P + 1] = lt1;
      out[P + 2] = lt2;
    }
  }
}

using VFn = void (*)(const float*, const int32_t*, const int32_t*, const int32_t*, const float*,
                     const int64_t*, const float*, const float*, const float*, float*, float*,
                     int64_t, int, int, int, int, int, float, float, int, int);

struct VEntry {
  int D, H1, H2;
  VFn fn[2];  // [loss]
  int GS, HS, TG, TH, ACC;
};

#define CNF_VJP(D, H1, H2)                                                                \
  {D, H1, H2, {k_vjp<D, H1, H2, false>, k_vjp<D, H1, H2, true>}, VS<D, H1, H2>::GS,      \
   VS<D, H1, H2>::HS, VS<D, H1, H2>::TG, VS<D, H1, H2>::TH, VS<D, H1, H2>::ACC}

const VEntry kVTable[] = {
#ifdef CNF_VJP_DEV  // development builds: the headline shape only
    CNF_VJP(10, 5, 5),
#else
    CNF_VJP(2, 5, 5), CNF_VJP(3, 5, 5), CNF_VJP(4, 5, 5), CNF_VJP(5, 5, 5), CNF_VJP(6, 5, 5),
    CNF_VJP(8, 5, 5), CNF_VJP(10, 5, 5), CNF_VJP(3, 3, 3), CNF_VJP(8, 3, 3), CNF_VJP(10, 3, 3),
    CNF_VJP(3, 3, 0), CNF_VJP(10, 10, 0), CNF_VJP(10, 10, 10), CNF_VJP(3, 0, 0),
    CNF_VJP(10, 0, 0), CNF_VJP(10, 7, 0), CNF_VJP(10, 5, 0), CNF_VJP(3, 5, 0),
#endif
};

const VEntry* find_entry(const Shape& s) {
  if (s.family != Family::kValu || s.strict) return nullptr;
  const int h1 = s.n_lin >= 2 ? s.units[1] : 0, h2 = s.n_lin >= 3 ? s.units[2] : 0;
  for (const auto& e : kVTable)
    if (e.D == s.D && e.H1 == h1 && e.H2 == h2) return &e;
  return nullptr;
}

size_t lds_bytes(const Shape& s, const VEntry& e) {
  return 4 * ((size_t)s.L * s.DT * kVRows + 16 * (size_t)(e.TG + e.TH) * kGP +
              (size_t)s.L * s.nets * e.ACC);
}

int64_t grid_for(int64_t B) {
  const int64_t nt = (B + kVRows - 1) / kVRows;
  return nt < kVGrid ? nt : kVGrid;
}

int partial_stride(const Shape& s) { return (int)(((s.layer_floats * s.L + 3) + 3) & ~3); }

using VFn2 = void (*)(const float*, const int32_t*, const int32_t*, const int32_t*, VArgs2);

struct V2Entry {
  int D, H1, H2;
  VFn2 fn[2][2][2];  // [nets - 1][loss][perm]
};

#define CNF_V2N(D, H1, H2, N)                                                        \
  {{k_vjp2<D, H1, H2, N, false, false>, k_vjp2<D, H1, H2, N, false, true>},          \
   {k_vjp2<D, H1, H2, N, true, false>, k_vjp2<D, H1, H2, N, true, true>}}
#define CNF_V2(D, H1, H2) {D, H1, H2, {CNF_V2N(D, H1, H2, 1), CNF_V2N(D, H1, H2, 2)}}

// the packed-SGPR shapes (cnf_sgpr.hip's table): every one has GS, HS <= 16
const V2Entry kV2Table[] = {
#ifdef CNF_VJP_DEV
    CNF_V2(10, 5, 5),
#else
    CNF_V2(2, 5, 5), CNF_V2(3, 5, 5), CNF_V2(4, 5, 5), CNF_V2(5, 5, 5),
    CNF_V2(6, 5, 5), CNF_V2(8, 5, 5), CNF_V2(10, 5, 5),
    CNF_V2(3, 3, 3), CNF_V2(8, 3, 3), CNF_V2(10, 3, 3),
    CNF_V2(3, 3, 0), CNF_V2(3, 0, 0), CNF_V2(10, 0, 0),
    CNF_V2(10, 5, 0), CNF_V2(3, 5, 0),
#endif
};

const V2Entry* find_v2(const Shape& s) {
  if (s.family != Family::kValu || s.strict || !s.sp_ok || !s.shift || s.L > kV2LMax)
    return nullptr;
  const int h1 = s.n_lin >= 2 ? s.units[1] : 0, h2 = s.n_lin >= 3 ? s.units[2] : 0;
  for (const auto& e : kV2Table)
    if (e.D == s.D && e.H1 == h1 && e.H2 == h2) return &e;
  return nullptr;
}

VFn2 pick_v2(const V2Entry* e, const Shape& s, bool loss) {
  return e->fn[s.scale ? 1 : 0][loss ? 1 : 0][s.any_perm ? 1 : 0];
}

size_t lds_v2(const Shape& s) { return (size_t)(kV2TR * s.D + 32 * kV2SS) * 4; }

// persistent grid: as many one-wave blocks as fit, at most one per tile
int64_t grid_v2(const Shape& s, VFn2 fn, int64_t B) {
  static std::mutex mu;
  static std::unordered_map<const void*, int> cache;
  int cap;
  {
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find((const void*)fn);
    if (it != cache.end()) {
      cap = it->second;
    } else {
      int n = 0, dev = 0, cus = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, 64, lds_v2(s)) != hipSuccess ||
          n < 1)
        n = 1;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
          cus < 1)
        cus = 256;
      cap = n * cus;
      cache[(const void*)fn] = cap;
    }
  }
  const int64_t nt = (B + kV2TR - 1) / kV2TR;
  return nt < cap ? nt : cap;
}

}  // namespace

int reduce_partials(const float* partials, int nblk, int PS, int P, float* grads, float* terms,
                    hipStream_t st) {
  if (P > 0) {
    // many records: a first pass folds chunks of R records into each chunk's
    // first record (in place), so enough blocks share the read; then the
    // chunk sums are added in order
    const unsigned cols = (unsigned)((P + 63) / 64);
    int nrec = nblk, stride = PS;
    if (nblk >= 128) {
      const int S = std::min(64, nblk / 32), R = (nblk + S - 1) / S;
      const int S2 = (nblk + R - 1) / R;
      float* part = const_cast<float*>(partials);
      hipLaunchKernelGGL(k_reduce_cols, dim3(cols, (unsigned)S2), dim3(256), 0, st, partials, nblk,
                         PS, P, part, R, (int64_t)R * PS);
      nrec = S2;
      stride = R * PS;
    }
    hipLaunchKernelGGL(k_reduce_cols, dim3(cols, 1), dim3(256), 0, st, partials, nrec, stride, P,
                       grads, nrec, (int64_t)0);
  }
  const bool r4 = PS == 4 && P == 0 && (reinterpret_cast<uintptr_t>(partials) & 15) == 0;
  if (terms && r4)
    hipLaunchKernelGGL(k_reduce_rows4, dim3(1), dim3(kRR), 0, st,
                       reinterpret_cast<const float4*>(partials), nblk, terms);
  else if (terms)
    hipLaunchKernelGGL(k_reduce_rows, dim3(1), dim3(64), 0, st, partials, nblk, PS, P, 3,
                       terms);
  return CNF_OK;
}

bool vjp2_ok(const Shape& s) { return find_v2(s) != nullptr; }

// workspace of k_vjp2: [per-wave partials][x_T stash], the stash 256-B aligned
size_t v2_stash_offset(const Shape& s, int64_t nblk) {
  return ((size_t)(nblk > 0 ? nblk : 1) * partial_stride(s) * 4 + 255) / 256 * 256;
}

int vjp_workspace(const Shape& s, int64_t B, size_t* bytes) {
  if (s.family == Family::kTile) return wvjp_workspace(s, B, bytes);
  if (!find_v2(s)) {  // narrow shapes outside both row-resident kernels
    const VEntry* e = find_entry(s);
    if (!e || lds_bytes(s, *e) > 64 * 1024) return wvjp_workspace(s, B, bytes);
  }
  if (const V2Entry* e2 = find_v2(s)) {
    // the larger of the two variants (loss / generic) -- same grid rule
    const int64_t g = std::max(grid_v2(s, pick_v2(e2, s, true), B),
                               grid_v2(s, pick_v2(e2, s, false), B));
    *bytes = v2_stash_offset(s, g) + (size_t)s.L * (B > 0 ? B : 1) * s.DT * 4;
    return CNF_OK;
  }
  const VEntry* e = find_entry(s);
  if (!e || lds_bytes(s, *e) > 64 * 1024) return CNF_ERR_UNSUPPORTED;
  *bytes = (size_t)(grid_for(B) > 0 ? grid_for(B) : 1) * partial_stride(s) * 4;
  return CNF_OK;
}

int vjp_run(const Shape& s, const void* prepared, const float* x, const int64_t* y,
            const float* gz, const float* gz_all, const float* gld, int kind, float det,
            float grad_scale, float* loss_terms, float* grads, float* dx, int64_t B, void* ws,
            size_t ws_bytes, hipStream_t st) {
  bool layerwise = s.family == Family::kTile;
  if (!layerwise && !find_v2(s)) {
    const VEntry* e = find_entry(s);
    layerwise = !e || lds_bytes(s, *e) > 64 * 1024;
  }
  if (layerwise)
    return wvjp_run(s, prepared, x, y, gz, gz_all, gld, kind, det, grad_scale, loss_terms, grads,
                    dx, B, ws, ws_bytes, st);
  if (const V2Entry* e2 = find_v2(s)) {
    size_t need = 0;
    int r = vjp_workspace(s, B, &need);
    if (r != CNF_OK) return r;
    if (!ws || ws_bytes < need) return CNF_ERR_NULL;
    const char* base = static_cast<const char*>(prepared);
    const int32_t* fq = reinterpret_cast<const int32_t*>(base);
    const int32_t* iq = fq + s.L * s.D;
    const int32_t* flags = iq + s.L * s.D;
    const float* W = reinterpret_cast<const float*>(base + idx_bytes(s)) + s.vp_region;
    VArgs2 a{};
    a.x = x;
    a.y = y;
    a.gz = gz;
    a.gz_all = gz_all;
    a.gld = gld;
    a.dx = dx;
    a.partials = static_cast<float*>(ws);
    const int64_t nblk = B > 0 ? grid_v2(s, pick_v2(e2, s, kind >= 0), B) : 0;
    const int64_t gmax = std::max(grid_v2(s, pick_v2(e2, s, true), B),
                                  grid_v2(s, pick_v2(e2, s, false), B));
    a.stash = reinterpret_cast<float*>(static_cast<char*>(ws) + v2_stash_offset(s, gmax));
    a.B = B;
    a.L = s.L;
    a.kind = kind;
    a.det = det;
    a.grad_scale = grad_scale;
    a.P = (int)(s.layer_floats * s.L);
    a.PS = partial_stride(s);
    const bool loss = kind >= 0;
    VFn2 fn = pick_v2(e2, s, loss);
    if (nblk > 0)
      hipLaunchKernelGGL(fn, dim3((unsigned)nblk), dim3(64), lds_v2(s), st, W, fq, iq, flags, a);
    reduce_partials(a.partials, (int)nblk, a.PS, a.P, grads, loss_terms, st);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
      set_hip_error(err);
      return CNF_ERR_HIP;
    }
    return CNF_OK;
  }
  const VEntry* e = find_entry(s);
  if (!e) return CNF_ERR_UNSUPPORTED;
  const size_t lds = lds_bytes(s, *e);
  if (lds > 64 * 1024) return CNF_ERR_UNSUPPORTED;
  size_t need = 0;
  int r = vjp_workspace(s, B, &need);
  if (r != CNF_OK) return r;
  if (!ws || ws_bytes < need) return CNF_ERR_NULL;
  const char* base = static_cast<const char*>(prepared);
  const int32_t* fq = reinterpret_cast<const int32_t*>(base);
  const int32_t* iq = fq + s.L * s.D;
  const int32_t* flags = iq + s.L * s.D;
  const float* W = reinterpret_cast<const float*>(base + idx_bytes(s));
  const int P = (int)(s.layer_floats * s.L);
  const int PS = partial_stride(s);
  float* partials = static_cast<float*>(ws);
  const int64_t nblk = grid_for(B);
  if (nblk > 0) {
    const bool loss = kind >= 0;
    hipLaunchKernelGGL(e->fn[loss ? 1 : 0], dim3((unsigned)nblk), dim3(kVRows), lds, st, W, fq,
                       iq, flags, x, y, gz, gz_all, gld, dx, partials, B, s.L, s.scale, s.shift,
                       s.any_perm ? 1 : 0, kind, det, grad_scale, P, PS);
  }
  reduce_partials(partials, (int)nblk, PS, P, grads, loss_terms, st);
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    set_hip_error(err);
    return CNF_ERR_HIP;
  }
  return CNF_OK;
}

}  // namespace cnf
