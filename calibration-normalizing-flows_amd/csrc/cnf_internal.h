// Internal declarations shared by the libcnf_hip translation units.
// Shapes are derived once from cnf_desc (include/cnf.h); every kernel family
// reads the same "prepared" blob prefix (index tables) followed by its own
// weight layout.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "cnf.h"

// roctx ranges around every launching C-ABI entry point (SURVEY.md section 5,
// tracing): compiled in only by `make roctx` (-DCNF_ROCTX, linked against
// rocprofiler-sdk-roctx; never the shipped build, which reads no environment
// and loads no tracer), so a `rocprofv3 --marker-trace --kernel-trace` run of
// that build ties each cnf_* host call to the kernels it launched.
#ifdef CNF_ROCTX
#include <rocprofiler-sdk-roctx/roctx.h>
namespace cnf {
struct RoctxRange {
  explicit RoctxRange(const char* name) { roctxRangePushA(name); }
  ~RoctxRange() { roctxRangePop(); }
};
}  // namespace cnf
#define CNF_RANGE(name) ::cnf::RoctxRange cnf_roctx_range_(name)
#else
#define CNF_RANGE(name) \
  do {                  \
  } while (0)
#endif

namespace cnf {

constexpr int kMaxLin = CNF_MAX_HIDDEN + 1;  // Linear layers per conditioner MLP

// Per-layer flags stored in the prepared blob.
constexpr int32_t kFlagPerm = 1;  // layer has a random_flip permutation

enum class Family { kValu, kTile };

// Host-side view of a descriptor.
struct Shape {
  int D = 0, DT = 0, DC = 0, L = 0;  // DT: transformed (mask 0), DC: conditioning (mask 1)
  int n_lin = 0;                     // Linear layers per net
  int units[kMaxLin + 1] = {};       // [D, h..., D]
  int scale = 1, shift = 1, strict = 0;
  int options = 0;                   // cnf_desc.options (CNF_OPT_*)
  bool alt_mask = false, s_tanh = false;  // legacy semantics (CNF_OPT_ALT_MASK / S_TANH)
  int nets = 2;                      // scale + shift
  int64_t net_floats = 0;            // natural layout (state_dict order)
  int64_t layer_floats = 0;
  bool any_perm = false;
  const int64_t* perms_host = nullptr;  // desc->perms (valid during the call)
  Family family = Family::kTile;
  int valu_id = -1;                  // index into the VALU instantiation table
  // VALU compact layout (cnf_valu_common.h): per Linear W[nout][pad4(nin)], b[pad4(nout)]
  int64_t valu_lin_off[kMaxLin] = {};
  int64_t valu_net_floats = 0;
  // pipelined-scalar layout (cnf_sgpr.hip), appended after the compact region:
  // per Linear W[nout][nin] + b[nout] (last Linear: nout = DT) padded to 16
  // floats; sp_ok when every Linear fits 32 floats
  bool sp_ok = false;
  int64_t sp_lin_off[kMaxLin] = {};
  int64_t sp_net_floats = 0;
  int64_t sp_region = 0;  // float offset of the region in the weights region
  int64_t vp_region = 0;  // the same layout with plain (unscaled) weights: reverse mode
  // tile (MFMA) layout
  int NO = 0;                        // last-linear outputs computed: DT (fast) or D (strict)
  int lin_nin[kMaxLin] = {}, lin_nout[kMaxLin] = {}, lin_inoff[kMaxLin] = {};
  int lin_OT[kMaxLin] = {}, lin_KS[kMaxLin] = {};
  int64_t tile_lin_off[kMaxLin] = {};  // float offset of linear i within a tiled net
  int64_t tile_net_floats = 0, tile_layer_floats = 0;
  int tile_hp = 0;                   // padded activation rows
  int tile_nop = 0;                  // padded S/T rows
  int tile_waves = 0;                // waves per block that fit LDS
  size_t tile_lds_bytes = 0;
  // register-resident MFMA layout (cnf_wide.hip), appended after the tile region
  int64_t wide_region = 0;           // float offset of the region in the weights region
  int64_t wide_floats = 0;           // floats of the region (0: shape not in its table)
  // natural (state_dict order) copy of every parameter, after the wide region:
  // the reverse mode's operands (cnf_wvjp.hip)
  int64_t plain_region = 0;
};

// Prepared blob: [int32 fwd_q L*D][int32 inv_q L*D][int32 flags L] padded to
// 256 B, then the weights region.
inline int64_t idx_bytes(const Shape& s) {
  int64_t b = (int64_t)(2 * s.L * s.D + s.L) * 4;
  return (b + 255) / 256 * 256;
}

int derive_shape(const cnf_desc* d, Shape* s);
void set_hip_error(hipError_t e);

// ---- kernel-family entry points (return cnf_status) ----
int valu_supported(const Shape& s);  // -> valu_id or -1
int valu_run(const Shape& s, const void* prepared, const float* in, float* out, float* ld,
             float* all, int64_t B, bool inverse, hipStream_t st, const int64_t* y = nullptr,
             float* loss_ws = nullptr, int kind = 0, float det = 0.f,
             float* loss_terms = nullptr);
int valu_loss_blocks(const Shape& s, int64_t B);  // per-block loss partials of the fused eval
bool sgpr_enabled(const Shape& s);
int64_t sgpr_blocks(const Shape& s, int64_t B);
// CNF_ERR_UNSUPPORTED when this launch needs k_valu (permuted loss/predict,
// misaligned batch views); log_priors != NULL: the fused predict pass
int sgpr_run(const Shape& s, const void* prepared, const float* in, float* out, float* ld,
             float* all, int64_t B, bool inverse, hipStream_t st, const int64_t* y,
             float* loss_ws, int kind, float det, float* loss_terms,
             const float* log_priors = nullptr);
// sum partials[b][i] over b in block order: grads[i] (i < P), terms[i - P] (i < P + 3)
int reduce_partials(const float* partials, int nblk, int PS, int P, float* grads, float* terms,
                    hipStream_t st);

int tile_configure(Shape* s);        // fills tile_* fields; CNF_OK or UNSUPPORTED
int tile_run(const Shape& s, const void* prepared, const float* in, float* out, float* ld,
             float* all, int64_t B, bool inverse, hipStream_t st);

int prepare_run(const Shape& s, const float* const* params, void* prepared, hipStream_t st);

int64_t wide_layer_floats(const Shape& s);  // 0 when the shape has no k_wide instance
bool wide_ok(const Shape& s);               // k_wide serves this descriptor's final outputs
int wide_prepare(const Shape& s, const float* const* params, void* prepared, hipStream_t st);
int wide_run(const Shape& s, const void* prepared, const float* in, float* out, float* ld,
             int64_t B, bool inverse, hipStream_t st, const float* log_priors = nullptr);
// Training of the wide stacks (cnf_wide16.hip): per-row tape / gradient
// layouts in floats (parts at -1 are absent).  Nets in natural order: 0 the
// s-net, 1 the t-net (one net: the t-net).  Every part is in slot order: unit
// u of a 16-unit tile sits at slot 16 (u >> 4) + 4 (u & 3) + ((u & 15) >> 2).
struct WTrain16Layout {
  int RW, GW;         // tape / gradient floats per row
  int xc, cw;         // conditioning half [x_C | 1], width
  int xt, s, ts;      // transformed half before the update, s-net output, width
  int h[2][3], hw[3]; // net n's hidden k (1..NL-1) [relu(h_k) | 1], width
  int glast[2];       // gradient of net n's output (width ts)
  int gpre[2][3], gpw[3];  // gradient of hidden k's pre-activation, width
};
// The tape and G arrays are wave-tiled: rows in blocks of 32 (allocated whole),
// a block's 32 x W floats as [W / 16 tiles][2][16 rows][16 slots] (row r =
// 32 w + 16 g + i, column c at w * 32 W + (c >> 4) * 512 + g * 256 + i * 16 +
// (c & 15)); one array of a layer is wide16_blocks(B) * 32 * W floats.
int wide16_train_layout(const Shape& s, WTrain16Layout* out);
inline int64_t wide16_blocks(int64_t B) { return (B + 31) / 32; }
// The loss seed fused into the forward sweep (null: the final output goes to
// zst / ld for k_wseed): per row the gradient of z_L (G, [B][D]) and of ld
// (gld), per 32-row wave the (loss, ce, ld) sums (part, 4 floats each).
struct WSeed16 {
  const int64_t* y;
  float* G;
  float* gld;
  float* part;
  float det, grad_scale;
  int kind;
};
// tbits: relu' bits, 512 words per 32 rows and layer (wide16_tbits_words)
int wide16_train_forward(const Shape& s, const void* prepared, const float* x, float* zst, int Cp,
                         int Dp, float* ld, float* tape, uint32_t* tbits, int64_t B,
                         const WSeed16* seed, hipStream_t st);
// the reverse sweep of every layer (one launch); gz: the seed (gradient of
// the last output), gz_all: [L][B][D] or null, dx: or null; gbuf: L x B x GW
int wide16_train_backward(const Shape& s, const void* prepared, const float* gz,
                          const float* gz_all, float* dx, const float* gld, const float* tape,
                          const uint32_t* tbits, float* gbuf, int64_t B, hipStream_t st);
inline int64_t wide16_tbits_words(int64_t B) { return (B + 31) / 32 * 512; }  // per layer
bool wide16_train_ok(const Shape& s);  // the fused training sweeps serve this descriptor
// the 16x16x4-tile implementation behind wide_* (cnf_wide16.hip)
int64_t wide16_layer_floats(const Shape& s);
int wide16_prepare(const Shape& s, const float* const* params, void* prepared, hipStream_t st);
int wide16_run(const Shape& s, const void* prepared, const float* in, float* out, float* ld,
               int64_t B, bool inverse, hipStream_t st, const float* log_priors);

// layer-at-a-time MFMA reverse mode of the tile family (cnf_wvjp.hip)
bool wvjp_ok(const Shape& s);
int wvjp_workspace(const Shape& s, int64_t B, size_t* bytes);
int wvjp_inv_workspace(const Shape& s, int64_t B, size_t* bytes);
int wvjp_run(const Shape& s, const void* prepared, const float* x, const int64_t* y,
             const float* gz, const float* gz_all, const float* gld, int kind, float det,
             float grad_scale, float* loss_terms, float* grads, float* dx, int64_t B, void* ws,
             size_t ws_bytes, hipStream_t st);

// reverse mode of the INVERSE transform (Flow.backward under autograd)
int wvjp_inv_run(const Shape& s, const void* prepared, const float* z, const float* gx,
                 const float* gx_all, const float* gld, float* grads, float* dz, int64_t B,
                 void* ws, size_t ws_bytes, hipStream_t st);

int vjp_workspace(const Shape& s, int64_t B, size_t* bytes);
bool vjp2_ok(const Shape& s);  // the packed-pair SGPR reverse-mode kernel serves this shape
// kind < 0: generic VJP from gz / gz_all / gld;  kind = CNF_LOSS_*: fused loss
int vjp_run(const Shape& s, const void* prepared, const float* x, const int64_t* y,
            const float* gz, const float* gz_all, const float* gld, int kind, float det,
            float grad_scale, float* loss_terms, float* grads, float* dx, int64_t B, void* ws,
            size_t ws_bytes, hipStream_t st);

}  // namespace cnf
