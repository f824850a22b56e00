// Dependent-issue microbenchmark (MI355X): v_pk_fma_f32 throughput per SIMD
// when each wave carries NCH independent FMA chains, at W waves per SIMD.
// Tells how much ILP a wave needs for the VALU to stay busy.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int NCH>
__global__ __launch_bounds__(256) void k(float* out, int iters) {
  f2 a[NCH];
#pragma unroll
  for (int i = 0; i < NCH; ++i) a[i] = f2{threadIdx.x * 1e-3f + i, i * 0.5f};
  const f2 x = f2{1.0001f, 0.9999f}, c = f2{1e-7f, 2e-7f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 48 / NCH; ++r)
#pragma unroll
      for (int i = 0; i < NCH; ++i) a[i] = __builtin_elementwise_fma(a[i], x, c);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NCH; ++i) s += a[i].x + a[i].y;
  if (s == 12345.f) out[threadIdx.x] = s;
}

template <int NCH>
void run(float* out, int cus, int waves_per_simd) {
  const int blocks = cus * waves_per_simd, iters = 4000;
  hipLaunchKernelGGL(k<NCH>, dim3(blocks), dim3(256), 0, 0, out, 10);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k<NCH>, dim3(blocks), dim3(256), 0, 0, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double instr = (double)blocks * 4 * iters * 48;  // wave-level pk_fma
  const double per_simd = instr / (cus * 4.0) / (ms * 1e-3);
  printf("{\"chains\": %d, \"waves_per_simd\": %d, \"pk_fma_per_simd_per_ns\": %.4f, \"cycles_per_pk_fma_at_2.4GHz\": %.2f}\n",
         NCH, waves_per_simd, per_simd * 1e-9, 2.4e9 / per_simd);
}

int main() {
  float* out;
  (void)hipMalloc(&out, 4096);
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  for (int w : {1, 2, 3, 4, 5, 8}) {
    run<1>(out, cus, w);
    run<2>(out, cus, w);
    run<4>(out, cus, w);
    run<8>(out, cus, w);
  }
  return 0;
}
