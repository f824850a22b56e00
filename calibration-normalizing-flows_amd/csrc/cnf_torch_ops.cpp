// torch.library binding of the coupling-flow engine: cnf::* operators
// registered from C++ (TORCH_LIBRARY), each a thin call of the C ABI in
// include/cnf.h on torch's current HIP stream, with outputs and workspaces from
// torch's (stream-aware) caching allocator.  `cnf::flow` carries an autograd
// kernel whose backward is cnf_vjp, so Flow.forward dispatches to one native
// launch per call without the Python ctypes path.
//
//   cnf::forward(x, prepared, desc, perms, inverse, all_outputs) -> (out, logdet)
//       Flow.forward / Flow.backward            flows/flows.py:17-37, 101-126
//   cnf::flow(x, prepared, desc, perms, all_outputs, params) -> (out, logdet)
//       the same forward with gradients for x and every parameter (autograd)
//   cnf::forward_loss(x, y, prepared, desc, perms, kind, det) -> terms[3]
//       TorchFlowCalibrator.fit eval sums      calibrators.py:297-317
//   cnf::loss_and_grads(x, y, prepared, desc, perms, kind, det, grad_scale) -> (terms, grads)
//       fused training step                    calibrators.py:284-295
//   cnf::vjp(x, prepared, desc, perms, gz, gz_all, gld, need_dx) -> (grads, dx)
//   cnf::inverse_flow(z, prepared, desc, perms, all_outputs, params) -> (out, logdet)
//       Flow.backward with gradients for z and every parameter (autograd;
//       backward = cnf_vjp_inverse)            flows/flows.py:27-37, 114-126
//   cnf::vjp_inverse(z, prepared, desc, perms, gx, gx_all, gld, need_dz) -> (grads, dz)
//   cnf::predict(x, prepared, desc, perms, log_priors) -> probs
//       Calibrator.predict                     calibrators.py:40-44, 330-353
//
// `desc` is the descriptor as integers: [dim, n_layers, n_hidden, hidden[0..7],
// scale, shift, strict_nan, options]; `perms` an optional host int64 [L, D]
// table (row[0] < 0: no permutation), as cnf_desc.perms.
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>
#include <torch/torch.h>

#include <vector>

#include "cnf.h"

namespace {

using torch::Tensor;
using torch::autograd::AutogradContext;
using torch::autograd::variable_list;

struct Desc {
  cnf_desc d{};
  Tensor perms;  // keeps the host table alive while d.perms points into it
};

Desc make_desc(c10::IntArrayRef v, const c10::optional<Tensor>& perms) {
  TORCH_CHECK(v.size() == 15, "cnf: desc must have 15 entries, got ", v.size());
  Desc r;
  r.d.abi_version = CNF_ABI_VERSION;
  r.d.dim = (int32_t)v[0];
  r.d.n_layers = (int32_t)v[1];
  r.d.n_hidden = (int32_t)v[2];
  for (int i = 0; i < CNF_MAX_HIDDEN; ++i) r.d.hidden[i] = (int32_t)v[3 + i];
  r.d.scale = (int32_t)v[11];
  r.d.shift = (int32_t)v[12];
  r.d.strict_nan = (int32_t)v[13];
  r.d.options = (int32_t)v[14];
  r.d.perms = nullptr;
  if (perms.has_value() && perms->defined()) {
    r.perms = perms->to(torch::kCPU, torch::kInt64).contiguous();
    TORCH_CHECK(r.perms.numel() == (int64_t)r.d.n_layers * r.d.dim, "cnf: perms must be [L, D]");
    r.d.perms = r.perms.data_ptr<int64_t>();
  }
  return r;
}

void check(const char* fn, int st) {
  TORCH_CHECK(st == CNF_OK, fn, " failed: ", cnf_strerror(st), " [", st, "]",
              st == CNF_ERR_HIP ? " (hipError " + std::to_string(cnf_last_hip_error()) + ")" : "");
}

// The current stream of x's device: the dispatcher sets no device guard for
// these operators, so each one guards x's device itself (DevGuard below) and
// launches on that device's current stream, as the ctypes path does.
void* stream(const Tensor& x) {
  return (void*)c10::hip::getCurrentHIPStream(x.device().index()).stream();
}
using DevGuard = c10::DeviceGuard;

const float* fptr(const c10::optional<Tensor>& t) {
  return t.has_value() && t->defined() ? t->data_ptr<float>() : nullptr;
}

Tensor rows(const Tensor& x, const Desc& d) {
  TORCH_CHECK(x.is_cuda(), "cnf: input must be a ROCm device tensor");
  TORCH_CHECK(x.scalar_type() == torch::kFloat32, "cnf: input must be fp32");
  TORCH_CHECK(x.dim() == 2 && x.size(1) == d.d.dim, "cnf: expected [B, ", d.d.dim, "] logits");
  return x.contiguous();
}

std::tuple<Tensor, Tensor> forward_impl(const Tensor& x_, const Tensor& prepared,
                                        c10::IntArrayRef desc, const c10::optional<Tensor>& perms,
                                        bool inverse, bool all_outputs) {
  DevGuard guard(x_.device());
  Desc d = make_desc(desc, perms);
  Tensor x = rows(x_, d);
  const int64_t B = x.size(0), D = d.d.dim, L = d.d.n_layers;
  Tensor ld = torch::empty({B}, x.options());
  Tensor out = all_outputs ? torch::empty({L, B, D}, x.options()) : torch::empty({B, D}, x.options());
  float* fin = all_outputs ? nullptr : out.data_ptr<float>();
  float* all = all_outputs ? out.data_ptr<float>() : nullptr;
  const int st = inverse ? cnf_inverse(&d.d, prepared.data_ptr(), x.data_ptr<float>(), fin,
                                       ld.data_ptr<float>(), all, B, stream(x))
                         : cnf_forward(&d.d, prepared.data_ptr(), x.data_ptr<float>(), fin,
                                       ld.data_ptr<float>(), all, B, stream(x));
  check(inverse ? "cnf_inverse" : "cnf_forward", st);
  return {out, ld};
}

Tensor forward_loss_impl(const Tensor& x_, const Tensor& y_, const Tensor& prepared,
                         c10::IntArrayRef desc, const c10::optional<Tensor>& perms, int64_t kind,
                         double det) {
  DevGuard guard(x_.device());
  Desc d = make_desc(desc, perms);
  Tensor x = rows(x_, d);
  Tensor y = y_.to(torch::kInt64).contiguous();
  const int64_t B = x.size(0);
  size_t n = 0;
  check("cnf_forward_loss_workspace_bytes", cnf_forward_loss_workspace_bytes(&d.d, B, &n));
  Tensor ws = torch::empty({(int64_t)std::max<size_t>(n, 16)}, x.options().dtype(torch::kUInt8));
  Tensor terms = torch::empty({3}, x.options());
  check("cnf_forward_loss",
        cnf_forward_loss(&d.d, prepared.data_ptr(), x.data_ptr<float>(), y.data_ptr<int64_t>(),
                         (int32_t)kind, (float)det, nullptr, nullptr, terms.data_ptr<float>(), B,
                         ws.data_ptr(), n, stream(x)));
  return terms;
}

int64_t param_count(const Desc& d) {
  int64_t n = 0;
  check("cnf_param_count", cnf_param_count(&d.d, &n));
  return n;
}

Tensor vjp_workspace(const Desc& d, int64_t B, const Tensor& like, size_t* n) {
  check("cnf_vjp_workspace_bytes", cnf_vjp_workspace_bytes(&d.d, B, n));
  return torch::empty({(int64_t)std::max<size_t>(*n, 16)}, like.options().dtype(torch::kUInt8));
}

std::tuple<Tensor, Tensor> loss_and_grads_impl(const Tensor& x_, const Tensor& y_,
                                               const Tensor& prepared, c10::IntArrayRef desc,
                                               const c10::optional<Tensor>& perms, int64_t kind,
                                               double det, double grad_scale) {
  DevGuard guard(x_.device());
  Desc d = make_desc(desc, perms);
  Tensor x = rows(x_, d);
  Tensor y = y_.to(torch::kInt64).contiguous();
  const int64_t B = x.size(0);
  size_t n = 0;
  Tensor ws = vjp_workspace(d, B, x, &n);
  Tensor terms = torch::empty({3}, x.options());
  Tensor grads = torch::empty({param_count(d)}, x.options());
  check("cnf_loss_vjp",
        cnf_loss_vjp(&d.d, prepared.data_ptr(), x.data_ptr<float>(), y.data_ptr<int64_t>(),
                     (int32_t)kind, (float)det, (float)grad_scale, terms.data_ptr<float>(),
                     grads.data_ptr<float>(), nullptr, B, ws.data_ptr(), n, stream(x)));
  return {terms, grads};
}

std::tuple<Tensor, Tensor> vjp_impl(const Tensor& x_, const Tensor& prepared,
                                    c10::IntArrayRef desc, const c10::optional<Tensor>& perms,
                                    const c10::optional<Tensor>& gz,
                                    const c10::optional<Tensor>& gz_all,
                                    const c10::optional<Tensor>& gld, bool need_dx) {
  DevGuard guard(x_.device());
  Desc d = make_desc(desc, perms);
  Tensor x = rows(x_, d);
  const int64_t B = x.size(0);
  auto cont = [](const c10::optional<Tensor>& t) -> c10::optional<Tensor> {
    if (!t.has_value() || !t->defined()) return c10::nullopt;
    return t->to(torch::kFloat32).contiguous();
  };
  c10::optional<Tensor> g1 = cont(gz), g2 = cont(gz_all), g3 = cont(gld);
  if (g3.has_value() && g3->numel() == 1 && B != 1) g3 = g3->reshape({1}).expand({B}).contiguous();
  size_t n = 0;
  Tensor ws = vjp_workspace(d, B, x, &n);
  Tensor grads = torch::empty({param_count(d)}, x.options());
  Tensor dx = need_dx ? torch::empty_like(x) : Tensor();
  check("cnf_vjp", cnf_vjp(&d.d, prepared.data_ptr(), x.data_ptr<float>(), fptr(g1), fptr(g2),
                           fptr(g3), grads.data_ptr<float>(),
                           need_dx ? dx.data_ptr<float>() : nullptr, B, ws.data_ptr(), n,
                           stream(x)));
  return {grads, dx};
}

std::tuple<Tensor, Tensor> vjp_inverse_impl(const Tensor& z_, const Tensor& prepared,
                                            c10::IntArrayRef desc,
                                            const c10::optional<Tensor>& perms,
                                            const c10::optional<Tensor>& gx,
                                            const c10::optional<Tensor>& gx_all,
                                            const c10::optional<Tensor>& gld, bool need_dz) {
  DevGuard guard(z_.device());
  Desc d = make_desc(desc, perms);
  Tensor z = rows(z_, d);
  const int64_t B = z.size(0);
  auto cont = [](const c10::optional<Tensor>& t) -> c10::optional<Tensor> {
    if (!t.has_value() || !t->defined()) return c10::nullopt;
    return t->to(torch::kFloat32).contiguous();
  };
  c10::optional<Tensor> g1 = cont(gx), g2 = cont(gx_all), g3 = cont(gld);
  if (g3.has_value() && g3->numel() == 1 && B != 1) g3 = g3->reshape({1}).expand({B}).contiguous();
  size_t n = 0;
  check("cnf_vjp_inverse_workspace_bytes", cnf_vjp_inverse_workspace_bytes(&d.d, B, &n));
  Tensor ws = torch::empty({(int64_t)std::max<size_t>(n, 16)}, z.options().dtype(torch::kUInt8));
  Tensor grads = torch::empty({param_count(d)}, z.options());
  Tensor dz = need_dz ? torch::empty_like(z) : Tensor();
  check("cnf_vjp_inverse",
        cnf_vjp_inverse(&d.d, prepared.data_ptr(), z.data_ptr<float>(), fptr(g1), fptr(g2),
                        fptr(g3), grads.data_ptr<float>(), need_dz ? dz.data_ptr<float>() : nullptr,
                        B, ws.data_ptr(), n, stream(z)));
  return {grads, dz};
}

Tensor predict_impl(const Tensor& x_, const Tensor& prepared, c10::IntArrayRef desc,
                    const c10::optional<Tensor>& perms, const Tensor& log_priors) {
  DevGuard guard(x_.device());
  Desc d = make_desc(desc, perms);
  Tensor x = rows(x_, d);
  Tensor lp = log_priors.to(x.device(), torch::kFloat32).contiguous();
  TORCH_CHECK(lp.numel() == d.d.dim, "cnf: log_priors must have ", d.d.dim, " entries");
  Tensor probs = torch::empty_like(x);
  check("cnf_predict", cnf_predict(&d.d, prepared.data_ptr(), x.data_ptr<float>(),
                                   lp.data_ptr<float>(), probs.data_ptr<float>(), nullptr,
                                   x.size(0), stream(x)));
  return probs;
}

// Autograd: forward = one fused launch, backward = cnf_vjp (recomputes the
// forward inside; nothing but x is saved).  INV: the inverse transform
// (Flow.backward), backward = cnf_vjp_inverse.
template <bool INV>
class FlowFnT : public torch::autograd::Function<FlowFnT<INV>> {
 public:
  static variable_list forward(AutogradContext* ctx, const Tensor& x, const Tensor& prepared,
                               c10::IntArrayRef desc, const c10::optional<Tensor>& perms,
                               bool all_outputs, at::TensorList params) {
    at::AutoDispatchBelowADInplaceOrView guard;
    auto [out, ld] = forward_impl(x, prepared, desc, perms, INV, all_outputs);
    ctx->save_for_backward({x, prepared});
    ctx->saved_data["desc"] = std::vector<int64_t>(desc.begin(), desc.end());
    ctx->saved_data["perms"] = perms.has_value() ? *perms : Tensor();
    ctx->saved_data["all"] = all_outputs;
    ctx->saved_data["nparams"] = (int64_t)params.size();
    std::vector<int64_t> versions;
    for (const Tensor& p : params) versions.push_back((int64_t)p._version());
    ctx->saved_data["versions"] = versions;
    ctx->saved_data["params"] = std::vector<Tensor>(params.begin(), params.end());
    return {out, ld};
  }

  static variable_list backward(AutogradContext* ctx, variable_list g) {
    // the prepared blob holds the forward's weights: a parameter written in
    // place since then would make these gradients disagree with torch's rule
    auto ps = ctx->saved_data["params"].toTensorVector();
    auto vs = ctx->saved_data["versions"].toIntVector();
    for (size_t i = 0; i < ps.size(); ++i)
      TORCH_CHECK(ps[i]._version() == (uint32_t)vs[i],
                  "one of the variables needed for gradient computation has been modified by an "
                  "inplace operation: a coupling-layer weight changed between the native forward "
                  "and its backward");
    auto saved = ctx->get_saved_variables();
    const Tensor& x = saved[0];
    const Tensor& prepared = saved[1];
    auto desc = ctx->saved_data["desc"].toIntVector();
    Tensor perms = ctx->saved_data["perms"].toTensor();
    const bool all = ctx->saved_data["all"].toBool();
    const bool need_dx = ctx->needs_input_grad(0);
    c10::optional<Tensor> gz, gza, gld;
    if (g[0].defined()) (all ? gza : gz) = g[0];
    if (g[1].defined()) gld = g[1];
    const c10::optional<Tensor> pm = perms.defined() ? c10::optional<Tensor>(perms) : c10::nullopt;
    auto [grads, dx] = INV ? vjp_inverse_impl(x, prepared, desc, pm, gz, gza, gld, need_dx)
                           : vjp_impl(x, prepared, desc, pm, gz, gza, gld, need_dx);
    variable_list out{dx, Tensor(), Tensor(), Tensor(), Tensor()};
    // the flat gradient (state_dict order) split and shaped per parameter
    int64_t off = 0;
    for (const Tensor& p : ps) {
      out.push_back(grads.narrow(0, off, p.numel()).view(p.sizes()));
      off += p.numel();
    }
    return out;
  }
};

template <bool INV>
std::tuple<Tensor, Tensor> flow_autograd(const Tensor& x, const Tensor& prepared,
                                         c10::IntArrayRef desc, const c10::optional<Tensor>& perms,
                                         bool all_outputs, const std::vector<Tensor>& params) {
  auto r = FlowFnT<INV>::apply(x, prepared, desc, perms, all_outputs, at::TensorList(params));
  return {r[0], r[1]};
}

template <bool INV>
std::tuple<Tensor, Tensor> flow_plain(const Tensor& x, const Tensor& prepared,
                                      c10::IntArrayRef desc, const c10::optional<Tensor>& perms,
                                      bool all_outputs, const std::vector<Tensor>&) {
  return forward_impl(x, prepared, desc, perms, INV, all_outputs);
}

}  // namespace

TORCH_LIBRARY(cnf, m) {
  m.def("forward(Tensor x, Tensor prepared, int[] desc, Tensor? perms, bool inverse, "
        "bool all_outputs) -> (Tensor, Tensor)");
  m.def("flow(Tensor x, Tensor prepared, int[] desc, Tensor? perms, bool all_outputs, "
        "Tensor[] params) -> (Tensor, Tensor)");
  m.def("forward_loss(Tensor x, Tensor y, Tensor prepared, int[] desc, Tensor? perms, int kind, "
        "float det) -> Tensor");
  m.def("loss_and_grads(Tensor x, Tensor y, Tensor prepared, int[] desc, Tensor? perms, "
        "int kind, float det, float grad_scale) -> (Tensor, Tensor)");
  m.def("vjp(Tensor x, Tensor prepared, int[] desc, Tensor? perms, Tensor? gz, Tensor? gz_all, "
        "Tensor? gld, bool need_dx) -> (Tensor, Tensor)");
  m.def("predict(Tensor x, Tensor prepared, int[] desc, Tensor? perms, Tensor log_priors) "
        "-> Tensor");
  m.def("inverse_flow(Tensor z, Tensor prepared, int[] desc, Tensor? perms, bool all_outputs, "
        "Tensor[] params) -> (Tensor, Tensor)");
  m.def("vjp_inverse(Tensor z, Tensor prepared, int[] desc, Tensor? perms, Tensor? gx, "
        "Tensor? gx_all, Tensor? gld, bool need_dz) -> (Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(cnf, CUDA, m) {
  m.impl("forward", forward_impl);
  m.impl("flow", flow_plain<false>);
  m.impl("inverse_flow", flow_plain<true>);
  m.impl("vjp_inverse", vjp_inverse_impl);
  m.impl("forward_loss", forward_loss_impl);
  m.impl("loss_and_grads", loss_and_grads_impl);
  m.impl("vjp", vjp_impl);
  m.impl("predict", predict_impl);
}

TORCH_LIBRARY_IMPL(cnf, Autograd, m) {
  m.impl("flow", flow_autograd<false>);
  m.impl("inverse_flow", flow_autograd<true>);
}
