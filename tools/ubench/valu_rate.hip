// VALU issue-rate microbenchmark (MI355X): how many wave-level VALU
// instructions per SIMD per second the hardware sustains for the instruction
// mixes of k_sgpr -- pure v_pk_fma_f32, pk_fma with 1 v_exp_f32 per 18 (the
// layer mix), and pk_fma with an SGPR operand re-aligned by s_mov (the weight
// path).  Prints one JSON line per mix.  Build: hipcc -O3 --offload-arch=gfx950
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int MIX>
__global__ __launch_bounds__(256, 5) void k(float* out, const float* __restrict__ w, int iters) {
  f2 a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = f2{threadIdx.x * 1e-3f + i, i * 0.5f};
  const f2 x = f2{1.0001f, 0.9999f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 18; ++r) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if constexpr (MIX == 2) {
          const float s = w[(r * 8 + i) & 63];  // SGPR weight operand
          a[i] = __builtin_elementwise_fma(f2(s), a[i], x);
        } else {
          a[i] = __builtin_elementwise_fma(a[i], x, f2{1e-7f, 1e-7f});
        }
      }
    }
    if constexpr (MIX == 1) {
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i].x = __builtin_amdgcn_exp2f(a[i].x * 1e-9f) + a[i].y;
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += a[i].x + a[i].y;
  if (s == 12345.f) out[threadIdx.x] = s;
}

int main() {
  float *out, *w;
  hipMalloc(&out, 4096);
  hipMalloc(&w, 4096);
  hipMemset(w, 0, 4096);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int blocks = cus * 5, iters = 2000;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  void (*fns[3])(float*, const float*, int) = {k<0>, k<1>, k<2>};
  const char* names[3] = {"pk_fma", "pk_fma+exp(1:18)", "pk_fma sgpr-weight"};
  for (int m = 0; m < 3; ++m) {
    hipLaunchKernelGGL(fns[m], dim3(blocks), dim3(256), 0, 0, out, w, 10);
    hipEventRecord(e0);
    hipLaunchKernelGGL(fns[m], dim3(blocks), dim3(256), 0, 0, out, w, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double waves = blocks * 4.0;
    const double per_wave = iters * (18.0 * 8 + (m == 1 ? 16 : 0));  // VALU per wave (approx)
    const double simds = cus * 4.0;
    const double rate = waves * per_wave / (ms * 1e-3) / simds;    // VALU / SIMD / s
    printf("{\"mix\": \"%s\", \"ms\": %.3f, \"valu_per_simd_per_s\": %.4e, \"cycles_per_valu_at_2.4GHz\": %.3f, \"pk_fma_tflops\": %.1f}\n",
           names[m], ms, rate, 2.4e9 / rate, waves * iters * 18.0 * 8 * 64 * 4 / (ms * 1e-3) / 1e12);
  }
  return 0;
}
