// Device-side non-finite guard (failure detection): the
// counterpart of the reference's NaN abort, run_experiment3D.py:129-131
//     if (preds != preds).any(): print('Aborting training due to nan values')
// without a host round trip.  cnf_guard_nonfinite ORs into a caller-owned
// int32:  1 if any element is NaN,  2 if any is +-inf.  The scan is an
// HBM-bound grid-stride pass (16-B loads when aligned); only a wave that
// found something issues one atomic OR, so a clean tensor costs no atomics.
// The flag is never cleared here: the caller zeroes it once and reads it
// whenever it likes (one flag can cover many launches, e.g. every batch of
// an epoch), so a training loop checks it without synchronising per step.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "cnf_internal.h"

namespace cnf {
namespace {

__device__ __forceinline__ int classify(float v) {
  return (v != v ? 1 : 0) | (__builtin_isinf(v) ? 2 : 0);
}

__global__ __launch_bounds__(256) void k_guard(const float* __restrict__ a, int64_t n, int vec,
                                               int32_t* __restrict__ flag) {
  int bits = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (vec) {
    const int64_t n4 = n / 4;
    using v4 = __attribute__((ext_vector_type(4))) float;
    const v4* a4 = reinterpret_cast<const v4*>(a);
    for (int64_t k = i; k < n4; k += stride) {
      const v4 q = __builtin_nontemporal_load(a4 + k);
      bits |= classify(q.x) | classify(q.y) | classify(q.z) | classify(q.w);
    }
    for (int64_t k = n4 * 4 + i; k < n; k += stride) bits |= classify(a[k]);
  } else {
    for (int64_t k = i; k < n; k += stride) bits |= classify(a[k]);
  }
  // one atomic per wave, and only when the wave saw a non-finite value
  const unsigned long long any = __ballot(bits != 0);
  if (any) {
    int w = bits;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) w |= __shfl_xor(w, o, 64);
    if ((threadIdx.x & 63) == 0) atomicOr(flag, w);
  }
}

}  // namespace
}  // namespace cnf

extern "C" int cnf_guard_nonfinite(const float* data, int64_t n, int32_t* flag, void* stream) {
  using namespace cnf;
  CNF_RANGE("cnf_guard_nonfinite");
  if (n < 0) return CNF_ERR_BATCH;
  if (!flag || (n > 0 && !data)) return CNF_ERR_NULL;
  if ((reinterpret_cast<uintptr_t>(data) & 3) || (reinterpret_cast<uintptr_t>(flag) & 3))
    return CNF_ERR_ALIGN;
  if (n == 0) return CNF_OK;
  const int vec = (reinterpret_cast<uintptr_t>(data) & 15) == 0;
  // enough waves to stream at HBM rate (256 CUs x 8 blocks), no more than the data needs
  const int64_t per_block = 256LL * (vec ? 16 : 4);
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(2048, (n + per_block - 1) / per_block));
  hipLaunchKernelGGL(k_guard, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, data, n,
                     vec, flag);
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    set_hip_error(err);
    return CNF_ERR_HIP;
  }
  return CNF_OK;
}
