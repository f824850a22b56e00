// extern "C" boundary of libcnf_hip.so (declared in include/cnf.h).
// Validates the descriptor, picks the kernel family, and forwards to it.
// No allocation, no host synchronisation, no global mutable state beyond the
// thread-local last-HIP-error slot.
#include <hip/hip_runtime.h>

#include "cnf_internal.h"

namespace cnf {

static thread_local int g_last_hip_error = 0;

void set_hip_error(hipError_t e) { g_last_hip_error = (int)e; }

int derive_shape(const cnf_desc* d, Shape* s) {
  if (!d || !s) return CNF_ERR_NULL;
  if (d->abi_version != CNF_ABI_VERSION) return CNF_ERR_DESC;
  if (d->dim < 2 || d->dim > CNF_MAX_DIM) return d->dim > CNF_MAX_DIM ? CNF_ERR_UNSUPPORTED
                                                                      : CNF_ERR_DESC;
  if (d->n_layers < 1 || d->n_hidden < 0 || d->n_hidden > CNF_MAX_HIDDEN) return CNF_ERR_DESC;
  if ((d->scale != 0 && d->scale != 1) || (d->shift != 0 && d->shift != 1)) return CNF_ERR_DESC;
  *s = Shape{};
  s->D = d->dim;
  s->DT = d->dim / 2;               // mask[:, dim//2:] = 1   (flows/flows.py:81-82)
  s->DC = d->dim - d->dim / 2;
  s->L = d->n_layers;
  s->scale = d->scale;
  s->shift = d->shift;
  s->strict = d->strict_nan ? 1 : 0;
  if (d->options & ~(CNF_OPT_NO_SGPR | CNF_OPT_NO_WIDE | CNF_OPT_ALT_MASK | CNF_OPT_S_TANH))
    return CNF_ERR_DESC;
  s->options = d->options;
  s->alt_mask = (d->options & CNF_OPT_ALT_MASK) != 0;
  s->s_tanh = (d->options & CNF_OPT_S_TANH) != 0;
  s->nets = d->scale + d->shift;
  s->n_lin = d->n_hidden + 1;       // units = [dim] + hidden + [dim]  (flows/utils.py:14)
  s->units[0] = d->dim;
  for (int i = 0; i < d->n_hidden; ++i) {
    if (d->hidden[i] < 1) return CNF_ERR_DESC;
    if (d->hidden[i] > CNF_MAX_WIDTH) return CNF_ERR_UNSUPPORTED;
    s->units[i + 1] = d->hidden[i];
  }
  s->units[s->n_lin] = d->dim;
  s->net_floats = 0;
  for (int i = 0; i < s->n_lin; ++i)
    s->net_floats += (int64_t)s->units[i + 1] * s->units[i] + s->units[i + 1];
  s->layer_floats = s->net_floats * s->nets;
  s->perms_host = d->perms;
  s->any_perm = false;
  if (d->perms) {
    for (int l = 0; l < s->L; ++l) {
      const int64_t* p = d->perms + (int64_t)l * s->D;
      if (p[0] < 0) continue;
      bool seen[CNF_MAX_DIM] = {};
      for (int j = 0; j < s->D; ++j) {
        if (p[j] < 0 || p[j] >= s->D || seen[p[j]]) return CNF_ERR_DESC;
        seen[p[j]] = true;
      }
      s->any_perm = true;
    }
  }
  if (s->alt_mask && s->any_perm) return CNF_ERR_DESC;
  // legacy semantics: k_valu (its tables' shapes, forward / inverse / eval) and
  // the MFMA-tile family; their reverse modes run layer at a time (cnf_wvjp)
  s->valu_id = s->D <= 16 ? valu_supported(*s) : -1;
  if (s->valu_id >= 0) {
    s->family = Family::kValu;
    int64_t off = 0;
    for (int i = 0; i < s->n_lin; ++i) {
      const int nin = i == 0 ? s->DC : s->units[i];
      const int nout = s->units[i + 1];
      s->valu_lin_off[i] = off;
      off += ((int64_t)nout * ((nin + 3) & ~3) + ((nout + 3) & ~3) + 15) & ~15;
    }
    s->valu_net_floats = off;
    s->sp_ok = true;
    off = 0;
    for (int i = 0; i < s->n_lin; ++i) {
      const int nin = i == 0 ? s->DC : s->units[i];
      const int nout = i == s->n_lin - 1 ? s->DT : s->units[i + 1];
      const int64_t f = ((int64_t)nout * ((nin + 2) & ~1) + 15) & ~15;  // cnf_sgpr.hip SP
      if (f > 32) s->sp_ok = false;
      s->sp_lin_off[i] = off;
      off += f;
    }
    s->sp_net_floats = off;
    s->sp_region = s->valu_net_floats * s->nets * s->L;
    s->vp_region = s->sp_region + s->sp_net_floats * s->nets * s->L;
    // natural copy for the layer-at-a-time reverse mode (shapes k_vjp2 / k_vjp
    // do not cover: L > 8, wide hidden layers)
    s->plain_region = s->sp_region + (s->sp_ok ? 2 * s->sp_net_floats * s->nets * s->L : 0);
  } else {
    s->family = Family::kTile;
    int st = tile_configure(s);
    if (st != CNF_OK) return st;
  }
  return CNF_OK;
}

}  // namespace cnf

using namespace cnf;

extern "C" {

int cnf_abi_version(void) { return CNF_ABI_VERSION; }

int cnf_last_hip_error(void) { return g_last_hip_error; }

const char* cnf_strerror(int status) {
  switch (status) {
    case CNF_OK: return "ok";
    case CNF_ERR_NULL: return "required pointer is NULL";
    case CNF_ERR_DESC: return "malformed cnf_desc";
    case CNF_ERR_UNSUPPORTED: return "shape outside every kernel's envelope";
    case CNF_ERR_BATCH: return "negative batch size";
    case CNF_ERR_HIP: return "HIP runtime error (see cnf_last_hip_error)";
    case CNF_ERR_ALIGN: return "pointer not 4-byte aligned";
    default: return "unknown cnf status";
  }
}

int cnf_param_count(const cnf_desc* desc, int64_t* n) {
  Shape s;
  int st = derive_shape(desc, &s);
  if (st != CNF_OK) return st;
  if (!n) return CNF_ERR_NULL;
  *n = s.layer_floats * s.L;
  return CNF_OK;
}

int cnf_param_tensor_count(const cnf_desc* desc, int32_t* n) {
  Shape s;
  int st = derive_shape(desc, &s);
  if (st != CNF_OK) return st;
  if (!n) return CNF_ERR_NULL;
  *n = s.L * s.nets * s.n_lin * 2;
  return CNF_OK;
}

int cnf_prepared_bytes(const cnf_desc* desc, size_t* bytes) {
  Shape s;
  int st = derive_shape(desc, &s);
  if (st != CNF_OK) return st;
  if (!bytes) return CNF_ERR_NULL;
  const int64_t wf = s.family == Family::kTile
                       ? s.tile_layer_floats * s.L + s.wide_floats + s.layer_floats * s.L
                       : s.valu_net_floats * s.nets * s.L +
                             (s.sp_ok ? 2 * s.sp_net_floats * s.nets * s.L : 0) +
                             s.layer_floats * s.L;
  // +256: scalar-cache prefetch reads whole 64-B lines past the last weight
  *bytes = (size_t)(idx_bytes(s) + wf * 4 + 256);
  return CNF_OK;
}

int cnf_prepare(const cnf_desc* desc, const float* const* params, void* prepared, void* stream) {
  CNF_RANGE("cnf_prepare");
  Shape s;
  int st = derive_shape(desc, &s);
  if (st != CNF_OK) return st;
  if (!prepared || (!params && s.nets > 0)) return CNF_ERR_NULL;
  return prepare_run(s, params, prepared, (hipStream_t)stream);
}

static int run(const cnf_desc* desc, const void* prepared, const float* in, float* out,
               float* ld, float* all, int64_t B, void* stream, bool inverse) {
  Shape s;
  int st = derive_shape(desc, &s);
  if (st != CNF_OK) return st;
  if (B < 0) return CNF_ERR_BATCH;
  if (B == 0) return CNF_OK;
  if (!prepared || !in || (!out && !all)) return CNF_ERR_NULL;
  auto mis = [](const void* p) { return p && (reinterpret_cast<uintptr_t>(p) & 3); };
  if (mis(in) || mis(out) || mis(ld) || mis(all)) return CNF_ERR_ALIGN;
  if (s.family == Family::kValu)
    return valu_run(s, prepared, in, out, ld, all, B, inverse, (hipStream_t)stream);
  return tile_run(s, prepared, in, out, ld, all, B, inverse, (hipStream_t)stream);
}

int cnf_forward(const cnf_desc* desc, const void* prepared, const float* x, float* z,
                float* logdet, float* z_all, int64_t B, void* stream) {
  CNF_RANGE("cnf_forward");
  return run(desc, prepared, x, z, logdet, z_all, B, stream, false);
}

int cnf_inverse(const cnf_desc* desc, const void* prepared, const float* z, float* x,
                float* logdet, float* x_all, int64_t B, void* stream) {
  CNF_RANGE("cnf_inverse");
  return run(desc, prepared, z, x, logdet, x_all, B, stream, true);
}

int cnf_forward_loss_workspace_bytes(const cnf_desc* desc, int64_t B, size_t* bytes) {
  Shape s;
  int st = derive_shape(desc, &s);
  if (st != CNF_OK) return st;
  if (!bytes) return CNF_ERR_NULL;
  if (B < 0) return CNF_ERR_BATCH;
  if (s.family != Family::kValu) return CNF_ERR_UNSUPPORTED;
  const int nb = B > 0 ? valu_loss_blocks(s, B) : 0;
  // [16 B reserved][per-block partials: 4 floats each]
  *bytes = (size_t)(1 + (nb > 0 ? nb : 1)) * 4 * sizeof(float);
  return CNF_OK;
}

int cnf_forward_loss(const cnf_desc* desc, const void* prepared, const float* x,
                     const int64_t* y, int32_t loss_kind, float det, float* z, float* logdet,
                     float* loss_terms, int64_t B, void* workspace, size_t workspace_bytes,
                     void* stream) {
  CNF_RANGE("cnf_forward_loss");
  Shape s;
  int st = derive_shape(desc, &s);
  if (st != CNF_OK) return st;
  if (B < 0) return CNF_ERR_BATCH;
  if (loss_kind != CNF_LOSS_CAL && loss_kind != CNF_LOSS_CE) return CNF_ERR_DESC;
  if (s.family != Family::kValu) return CNF_ERR_UNSUPPORTED;
  if (!prepared || !loss_terms || (B > 0 && (!x || !y))) return CNF_ERR_NULL;
  size_t need = 0;
  st = cnf_forward_loss_workspace_bytes(desc, B, &need);
  if (st != CNF_OK) return st;
  if (!workspace || workspace_bytes < need) return CNF_ERR_NULL;
  auto mis = [](const void* p) { return p && (reinterpret_cast<uintptr_t>(p) & 3); };
  if (mis(x) || mis(z) || mis(logdet)) return CNF_ERR_ALIGN;
  float* ws = static_cast<float*>(workspace);
  if (B > 0) {
    st = valu_run(s, prepared, x, z, logdet, nullptr, B, false, (hipStream_t)stream, y, ws,
                  loss_kind, det, loss_terms);
    if (st != CNF_OK) return st;
  } else {
    hipError_t e = hipMemsetAsync(loss_terms, 0, 3 * sizeof(float), (hipStream_t)stream);
    if (e != hipSuccess) {
      set_hip_error(e);
      return CNF_ERR_HIP;
    }
  }
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    set_hip_error(err);
    return CNF_ERR_HIP;
  }
  return CNF_OK;
}

int cnf_predict(const cnf_desc* desc, const void* prepared, const float* x,
                const float* log_priors, float* probs, float* logdet, int64_t B, void* stream) {
  CNF_RANGE("cnf_predict");
  Shape s;
  int st = derive_shape(desc, &s);
  if (st != CNF_OK) return st;
  if (B < 0) return CNF_ERR_BATCH;
  const bool narrow = s.family == Family::kValu && sgpr_enabled(s);
  const bool wide = s.family == Family::kTile && s.wide_floats > 0 && wide_ok(s);
  if (!narrow && !wide) return CNF_ERR_UNSUPPORTED;
  if (B == 0) return CNF_OK;
  if (!prepared || !x || !log_priors || !probs) return CNF_ERR_NULL;
  auto mis = [](const void* p) { return p && (reinterpret_cast<uintptr_t>(p) & 3); };
  if (mis(x) || mis(probs) || mis(logdet) || mis(log_priors)) return CNF_ERR_ALIGN;
  if (wide)  // k_wide's predict mode (centre + flow + softmax + prior correction)
    return wide_run(s, prepared, x, probs, logdet, B, false, (hipStream_t)stream, log_priors);
  return sgpr_run(s, prepared, x, probs, logdet, nullptr, B, false, (hipStream_t)stream, nullptr,
                  nullptr, 0, 0.f, nullptr, log_priors);
}

int cnf_vjp_workspace_bytes(const cnf_desc* desc, int64_t B, size_t* bytes) {
  Shape s;
  int st = derive_shape(desc, &s);
  if (st != CNF_OK) return st;
  if (!bytes) return CNF_ERR_NULL;
  if (B < 0) return CNF_ERR_BATCH;
  return vjp_workspace(s, B, bytes);
}

int cnf_vjp(const cnf_desc* desc, const void* prepared, const float* x, const float* gz,
            const float* gz_all, const float* gld, float* grads, float* dx, int64_t B,
            void* workspace, size_t workspace_bytes, void* stream) {
  CNF_RANGE("cnf_vjp");
  Shape s;
  int st = derive_shape(desc, &s);
  if (st != CNF_OK) return st;
  if (B < 0) return CNF_ERR_BATCH;
  if (!prepared || !grads || (B > 0 && !x)) return CNF_ERR_NULL;
  return vjp_run(s, prepared, x, nullptr, gz, gz_all, gld, -1, 0.f, 1.f, nullptr, grads, dx, B,
                 workspace, workspace_bytes, (hipStream_t)stream);
}

int cnf_loss_vjp(const cnf_desc* desc, const void* prepared, const float* x, const int64_t* y,
                 int32_t loss_kind, float det, float grad_scale, float* loss_terms, float* grads,
                 float* dx, int64_t B, void* workspace, size_t workspace_bytes, void* stream) {
  CNF_RANGE("cnf_loss_vjp");
  Shape s;
  int st = derive_shape(desc, &s);
  if (st != CNF_OK) return st;
  if (B < 0) return CNF_ERR_BATCH;
  if (loss_kind != CNF_LOSS_CAL && loss_kind != CNF_LOSS_CE) return CNF_ERR_DESC;
  if (!prepared || !loss_terms || !grads || (B > 0 && (!x || !y))) return CNF_ERR_NULL;
  return vjp_run(s, prepared, x, y, nullptr, nullptr, nullptr, loss_kind, det, grad_scale,
                 loss_terms, grads, dx, B, workspace, workspace_bytes, (hipStream_t)stream);
}

int cnf_vjp_inverse_workspace_bytes(const cnf_desc* desc, int64_t B, size_t* bytes) {
  Shape s;
  int st = derive_shape(desc, &s);
  if (st != CNF_OK) return st;
  if (!bytes) return CNF_ERR_NULL;
  if (B < 0) return CNF_ERR_BATCH;
  return wvjp_inv_workspace(s, B, bytes);
}

int cnf_vjp_inverse(const cnf_desc* desc, const void* prepared, const float* z, const float* gx,
                    const float* gx_all, const float* gld, float* grads, float* dz, int64_t B,
                    void* workspace, size_t workspace_bytes, void* stream) {
  CNF_RANGE("cnf_vjp_inverse");
  Shape s;
  int st = derive_shape(desc, &s);
  if (st != CNF_OK) return st;
  if (B < 0) return CNF_ERR_BATCH;
  if (!prepared || !grads || (B > 0 && !z)) return CNF_ERR_NULL;
  return wvjp_inv_run(s, prepared, z, gx, gx_all, gld, grads, dz, B, workspace, workspace_bytes,
                      (hipStream_t)stream);
}

const char* cnf_kernel_name(const cnf_desc* desc) {
  Shape s;
  if (derive_shape(desc, &s) != CNF_OK) return "unsupported";
  if (s.family != Family::kValu)
    return s.wide_floats > 0 && wide_ok(s) ? "mfma-wide" : "mfma-tile";
  return sgpr_enabled(s) ? "sgpr-fused" : "valu-fused";
}

}  // extern "C"
