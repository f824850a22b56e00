// One-launch Adam step over every parameter of a coupling stack, fed by the
// flat gradient cnf_loss_vjp writes (state_dict order): the on-device
// optimizer of the calibrator's training step (the
// reference steps torch.optim.Adam, calibrators.py:239-295, at its defaults).
//
// Per element, as torch.optim.Adam's single-tensor update (amsgrad off):
//   g  = grad + weight_decay * p
//   m  = m + (1 - beta1) * (g - m)                (exp_avg.lerp_(g, 1 - beta1))
//   v  = beta2 * v + (1 - beta2) * g * g          (exp_avg_sq.mul_().addcmul_())
//   p -= lr / (1 - beta1^t) * m / (sqrt(v) / sqrt(1 - beta2^t) + eps)
// The moments live in two flat device buffers the caller owns (cnf_param_count
// floats each, zero before the first step).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

#include "cnf_internal.h"

namespace cnf {
namespace {

constexpr int kAdamTensors = 128;  // parameter tensors per launch (kernel-argument table)

struct AdamArgs {
  float* p[kAdamTensors];
  int64_t off[kAdamTensors + 1];  // flat offset of each tensor, and the end
  const float* g;
  float* m;
  float* v;
  // torch's scalars, each rounded to fp32 once: 1 - beta1 and 1 - beta2 are
  // formed in double from the optimizer's Python floats (torch/optim/adam.py
  // _single_tensor_adam: lerp_(grad, 1 - beta1), addcmul_(value=1 - beta2))
  float omb1, beta2, omb2, eps, wd, step_size, bc2_sqrt;
  // device {step_size, bc2_sqrt} (cnf_adam_step_sched: graph-captured steps,
  // whose kernel arguments are fixed at capture); nullptr: the two above
  const float* sched;
  // device int32 flag (cnf_adam_step_guarded): non-zero skips the whole update,
  // so a step whose gradient tripped the non-finite guard leaves the
  // parameters and moments at the last finite step; nullptr: always update
  const int32_t* skip;
};

__global__ __launch_bounds__(256) void k_adam(AdamArgs a) {
  if (a.skip && __builtin_amdgcn_readfirstlane(*a.skip) != 0) return;
  const int ti = blockIdx.y;
  const int64_t o0 = a.off[ti], n = a.off[ti + 1] - o0;
  float* __restrict__ p = a.p[ti];
  const float step_size = a.sched ? a.sched[0] : a.step_size;
  const float bc2_sqrt = a.sched ? a.sched[1] : a.bc2_sqrt;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t f = o0 + i;
    const float pv = p[i];
    // torch's operation order, each product rounded on its own
    float g = a.g[f];
    if (a.wd != 0.f) g = __fadd_rn(g, __fmul_rn(a.wd, pv));            // grad.add(p, alpha=wd)
    float m = a.m[f];
    m = __fadd_rn(m, __fmul_rn(a.omb1, __fsub_rn(g, m)));              // lerp_(g, 1 - beta1)
    const float v = __fadd_rn(__fmul_rn(a.v[f], a.beta2),
                              __fmul_rn(__fmul_rn(g, g), a.omb2));         // mul_().addcmul_()
    a.m[f] = m;
    a.v[f] = v;
    const float denom = __fadd_rn(__fdiv_rn(sqrtf(v), bc2_sqrt), a.eps);
    p[i] = __fadd_rn(pv, __fmul_rn(-step_size, __fdiv_rn(m, denom)));    // addcdiv_
  }
}

}  // namespace
}  // namespace cnf

using namespace cnf;

namespace {

int adam_launch(const cnf_desc* desc, float* const* params, const float* grads, float* exp_avg,
                float* exp_avg_sq, int64_t step, double lr, double beta1, double beta2, double eps,
                double weight_decay, const float* sched, const int32_t* skip, void* stream) {
  Shape s;
  int st = derive_shape(desc, &s);
  if (st != CNF_OK) return st;
  if (!sched && step < 1) return CNF_ERR_DESC;
  const int nt = s.L * s.nets * s.n_lin * 2;
  if (nt == 0) return CNF_OK;
  if (!params || !grads || !exp_avg || !exp_avg_sq) return CNF_ERR_NULL;
  const double bc1 = sched ? 1.0 : 1.0 - std::pow(beta1, (double)step);
  const double bc2 = sched ? 1.0 : 1.0 - std::pow(beta2, (double)step);
  AdamArgs a{};
  a.sched = sched;
  a.skip = skip;
  a.g = grads;
  a.m = exp_avg;
  a.v = exp_avg_sq;
  a.omb1 = (float)(1.0 - beta1);
  a.beta2 = (float)beta2;
  a.omb2 = (float)(1.0 - beta2);
  a.eps = (float)eps;
  a.wd = (float)weight_decay;
  a.step_size = (float)(lr / bc1);
  a.bc2_sqrt = (float)std::sqrt(bc2);
  // tensor sizes in ABI order: per layer, per net, per Linear: W then b
  int64_t off = 0;
  int k = 0, first = 0;
  auto flush = [&](int n_here) {
    if (n_here == 0) return;
    int64_t maxn = 0;
    for (int i = 0; i < n_here; ++i) maxn = std::max(maxn, a.off[i + 1] - a.off[i]);
    const unsigned gx = (unsigned)std::min<int64_t>((maxn + 255) / 256, 64);
    hipLaunchKernelGGL(k_adam, dim3(gx, (unsigned)n_here), dim3(256), 0, (hipStream_t)stream, a);
  };
  for (int l = 0; l < s.L; ++l)
    for (int n = 0; n < s.nets; ++n)
      for (int i = 0; i < s.n_lin; ++i)
        for (int wb = 0; wb < 2; ++wb) {
          const int64_t cnt = wb == 0 ? (int64_t)s.units[i + 1] * s.units[i] : s.units[i + 1];
          float* p = params[first + k];
          if (!p) return CNF_ERR_NULL;
          a.p[k] = p;
          a.off[k] = off;
          off += cnt;
          a.off[k + 1] = off;
          if (++k == kAdamTensors) {
            // offsets of the next chunk restart from its first tensor's position
            flush(k);
            first += k;
            const int64_t base = off;
            k = 0;
            a.off[0] = base;
          }
        }
  flush(k);
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    set_hip_error(err);
    return CNF_ERR_HIP;
  }
  return CNF_OK;
}

}  // namespace

extern "C" int cnf_adam_step(const cnf_desc* desc, float* const* params, const float* grads,
                             float* exp_avg, float* exp_avg_sq, int64_t step, double lr,
                             double beta1, double beta2, double eps, double weight_decay,
                             void* stream) {
  CNF_RANGE("cnf_adam_step");
  return adam_launch(desc, params, grads, exp_avg, exp_avg_sq, step, lr, beta1, beta2, eps,
                     weight_decay, nullptr, nullptr, stream);
}

extern "C" int cnf_adam_step_sched(const cnf_desc* desc, float* const* params,
                                   const float* grads, float* exp_avg, float* exp_avg_sq,
                                   const float* sched, double beta1, double beta2, double eps,
                                   double weight_decay, void* stream) {
  CNF_RANGE("cnf_adam_step_sched");
  if (!sched) return CNF_ERR_NULL;
  return adam_launch(desc, params, grads, exp_avg, exp_avg_sq, 0, 0.0, beta1, beta2, eps,
                     weight_decay, sched, nullptr, stream);
}

extern "C" int cnf_adam_step_guarded(const cnf_desc* desc, float* const* params,
                                     const float* grads, float* exp_avg, float* exp_avg_sq,
                                     int64_t step, double lr, const float* sched, double beta1,
                                     double beta2, double eps, double weight_decay,
                                     const int32_t* skip_flag, void* stream) {
  CNF_RANGE("cnf_adam_step_guarded");
  if (!skip_flag) return CNF_ERR_NULL;
  return adam_launch(desc, params, grads, exp_avg, exp_avg_sq, step, lr, beta1, beta2, eps,
                     weight_decay, sched, skip_flag, stream);
}
