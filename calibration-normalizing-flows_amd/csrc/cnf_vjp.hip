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
#include "cnf_valu_io.h"
#include "cnf_vjp2.h"

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

using v2::wave_sync;  // cnf_vjp2.h

// One MLP forward keeping its activations (compact weights, cnf_valu_common.h).
template <int D, int H1, int H2>
__device__ __forceinline__ void mlp_keep(const float* __restrict__ w, const float* c, float* h1,
                                         float* h2, float* out) {
  constexpr int DT = D / 2, DC = D - D / 2;
  if constexpr (H1 == 0) {
    linear<DC, D, DT, 0, false, false>(w, c, out, 0.f);
  } else if constexpr (H2 == 0) {
    linear<DC, H1, H1, 1, false, false>(w, c, h1, 0.f);
    linear<H1, D, DT, 0, false, false>(w + Lin<DC, H1>::floats, h1, out, 0.f);
  } else {
    linear<DC, H1, H1, 1, false, false>(w, c, h1, 0.f);
    const float* w2 = w + Lin<DC, H1>::floats;
    linear<H1, H2, H2, 1, false, false>(w2, h1, h2, 0.f);
    linear<H2, D, DT, 0, false, false>(w2 + Lin<H1, H2>::floats, h2, out, 0.f);
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
    for (int m = 0; m < H1; ++m) gh1[m] = h1[m] <= 0.f ? 0.f : gh1[m];
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
    for (int k = 0; k < H2; ++k) gh2[k] = h2[k] <= 0.f ? 0.f : gh2[k];
    linear_t<H1, H2, H2>(w2, gh2, gh1);
#pragma unroll
    for (int m = 0; m < H1; ++m) gh1[m] = h1[m] <= 0.f ? 0.f : gh1[m];
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
// reads).  grid.y = 1 gives the final sums; columns from `split` on then go to
// out2 (the loss sums that follow the gradients in each record), so one pass
// serves both.  Fixed grouping: deterministic.
__global__ __launch_bounds__(256) void k_reduce_cols(const float* __restrict__ partials, int nblk,
                                                     int PS, int NE, float* __restrict__ out,
                                                     int R, int64_t ostride,
                                                     float* __restrict__ out2, int split) {
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
  if (g == 0 && e < NE) {
    const float v = ((red[threadIdx.x] + red[threadIdx.x + 64]) + red[threadIdx.x + 128]) +
                    red[threadIdx.x + 192];
    if (e >= split) out2[e - split] = v;
    else out[(int64_t)blockIdx.y * ostride + e] = v;
  }
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
// forward-loss kernels' layout): one block, cnf_valu_io.h reduce_rows4_block.
using valu::kRR;
__global__ __launch_bounds__(kRR) void k_reduce_rows4(const float4* __restrict__ partials,
                                                      int nblk, float* __restrict__ out) {
  __shared__ float red[kRR / 64][3];
  valu::reduce_rows4_block(partials, nblk, out, red);
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
  if (s.family != Family::kValu || s.strict || s.alt_mask || s.s_tanh) return nullptr;
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

using v2::kV2TR;
using v2::kV2LMax;
using v2::kV2SS;

const V2Entry* find_v2(const Shape& s) {
  if (s.family != Family::kValu || s.strict || !s.sp_ok || !s.shift || s.L > kV2LMax ||
      s.alt_mask || s.s_tanh)
    return nullptr;
  const int h1 = s.n_lin >= 2 ? s.units[1] : 0, h2 = s.n_lin >= 3 ? s.units[2] : 0;
  const V2Entry* parts[3] = {kV2PartA, kV2PartB, kV2PartC};
  const int nums[3] = {kV2PartANum, kV2PartBNum, kV2PartCNum};
  for (int q = 0; q < 3; ++q)
    for (int i = 0; i < nums[q]; ++i) {
      const V2Entry& e = parts[q][i];
      if (e.D == s.D && e.H1 == h1 && e.H2 == h2) return &e;
    }
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
    // chunk sums are added in order.  The loss sums (columns P..P+2 of each
    // record, when asked for) ride the same passes.
    const int NE = terms ? P + 3 : P;
    const unsigned cols = (unsigned)((NE + 63) / 64);
    int nrec = nblk, stride = PS;
    if (nblk >= 128) {
      const int S = std::min(64, nblk / 32), R = (nblk + S - 1) / S;
      const int S2 = (nblk + R - 1) / R;
      float* part = const_cast<float*>(partials);
      hipLaunchKernelGGL(k_reduce_cols, dim3(cols, (unsigned)S2), dim3(256), 0, st, partials, nblk,
                         PS, NE, part, R, (int64_t)R * PS, (float*)nullptr, NE);
      nrec = S2;
      stride = R * PS;
    }
    hipLaunchKernelGGL(k_reduce_cols, dim3(cols, 1), dim3(256), 0, st, partials, nrec, stride, NE,
                       grads, nrec, (int64_t)0, terms, P);
    return CNF_OK;
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
    // the stash: L x DT x (B rounded up to even) floats (k_vjp2's pair stores)
    *bytes = v2_stash_offset(s, g) + (size_t)s.L * (((B > 0 ? B : 1) + 1) & ~(int64_t)1) * s.DT * 4;
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
