// Fused forward + loss + reverse-mode kernel (training path).  Placeholder
// until the VJP kernels land: reports CNF_ERR_UNSUPPORTED.
#include <hip/hip_runtime.h>

#include "cnf_internal.h"

namespace cnf {

int vjp_workspace(const Shape& s, int64_t B, size_t* bytes) {
  (void)s;
  (void)B;
  *bytes = 0;
  return CNF_ERR_UNSUPPORTED;
}

int vjp_run(const Shape& s, const void* prepared, const float* x, const int64_t* y, int kind,
            float det, float grad_scale, float* loss_terms, float* grads, float* dx, int64_t B,
            void* ws, size_t ws_bytes, hipStream_t st) {
  (void)s; (void)prepared; (void)x; (void)y; (void)kind; (void)det; (void)grad_scale;
  (void)loss_terms; (void)grads; (void)dx; (void)B; (void)ws; (void)ws_bytes; (void)st;
  return CNF_ERR_UNSUPPORTED;
}

}  // namespace cnf
