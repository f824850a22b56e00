// Micro-benchmark: sustained VALU FMA rate on this GPU (v_fma_f32 with VGPR /
// SGPR operands, v_pk_fma_f32), to pin the VALU ceiling the coupling kernel
// is measured against.  Build: hipcc -O3 --offload-arch=gfx950 valu_peak.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int NACC>
__global__ __launch_bounds__(256) void k_fma_v(float* out, float s0, int iters) {
  float a[NACC];
  float x = threadIdx.x * 1e-3f, y = 1.0001f;
#pragma unroll
  for (int i = 0; i < NACC; ++i) a[i] = x + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) a[i] = fmaf(a[i], y, x);
  }
  float r = 0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) r += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

// weight operand from an SGPR (wave-uniform), like the coupling kernel
template <int NACC>
__global__ __launch_bounds__(256) void k_fma_s(float* out, const float* __restrict__ w, int iters) {
  float a[NACC];
  float x = threadIdx.x * 1e-3f;
#pragma unroll
  for (int i = 0; i < NACC; ++i) a[i] = x + i;
  for (int it = 0; it < iters; ++it) {
    const float s = w[it & 15];
#pragma unroll
    for (int i = 0; i < NACC; ++i) a[i] = fmaf(s, a[i], x);
  }
  float r = 0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) r += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int NACC>
__global__ __launch_bounds__(256) void k_pk(float* out, float s0, int iters) {
  f2 a[NACC];
  f2 x = {threadIdx.x * 1e-3f, 0.5f}, y = {1.0001f, 0.9999f};
#pragma unroll
  for (int i = 0; i < NACC; ++i) a[i] = x + (float)i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) a[i] = __builtin_elementwise_fma(a[i], y, x);
  }
  f2 r = {0, 0};
#pragma unroll
  for (int i = 0; i < NACC; ++i) r += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r.x + r.y;
}

template <class K>
double run(K kern, const char* name, int blocks, int iters, double flops_per_thread_iter,
           float* out, const float* w, bool use_w) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep) {
    hipEventRecord(e0);
    if (use_w)
      hipLaunchKernelGGL((void (*)(float*, const float*, int))kern, dim3(blocks), dim3(256), 0, 0, out, w, iters);
    else
      hipLaunchKernelGGL((void (*)(float*, float, int))kern, dim3(blocks), dim3(256), 0, 0, out, 1.0f, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
  }
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  double tf = (double)blocks * 256 * iters * flops_per_thread_iter / (ms * 1e-3) / 1e12;
  printf("%-28s blocks=%5d  %8.3f ms  %7.1f TFLOP/s\n", name, blocks, ms, tf);
  return tf;
}

int main() {
  float* out;
  float* w;
  hipMalloc(&out, 256 * 8192 * 4 * sizeof(float));
  hipMalloc(&w, 64 * sizeof(float));
  hipMemset(w, 0, 64 * sizeof(float));
  const int iters = 4096;
  for (int blocks : {1024, 2048, 8192}) {
    run((const void*)k_fma_v<8>, "v_fma_f32 8 acc", blocks, iters, 16.0, out, w, false);
    run((const void*)k_fma_v<16>, "v_fma_f32 16 acc", blocks, iters, 32.0, out, w, false);
    run((const void*)k_fma_s<16>, "v_fma_f32 sgpr 16 acc", blocks, iters, 32.0, out, w, true);
    run((const void*)k_pk<8>, "v_pk_fma_f32 8 acc", blocks, iters, 32.0, out, w, false);
  }
  return 0;
}
