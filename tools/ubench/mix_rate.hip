// Micro-benchmark: can fp32 MFMA work run BESIDE a packed-fp32 VALU stream on
// one SIMD, and what does each MFMA cost the VALU issue?  (The narrow
// coupling kernels are VALU-bound; the f32 MFMA pipe is a second pipe of the
// same peak rate.)  Each wave runs ITERS iterations of NV v_pk_fma_f32 (8
// independent accumulators, SGPR weight operand as in k_sgpr) and NM MFMAs
// (MT 0: v_mfma_f32_4x4x1_16b_f32, 1: v_mfma_f32_16x16x4_f32; 4 independent
// accumulators), or NU plain v_fma_f32.  W waves per SIMD (one 256-thread block
// per CU per wave slot).  Cycles from s_memtime inside the kernel.
// Build: hipcc -O3 --offload-arch=gfx950 -o mix_rate mix_rate.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f2 pkfma(f2 w, f2 x, f2 acc) {
  f2 a;
  asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]" : "=v"(a) : "s"(w), "v"(x), "v"(acc));
  return a;
}
__device__ __forceinline__ void mfma4(v4f& acc, float a, float b) {
  asm volatile("v_mfma_f32_4x4x1_16b_f32 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma16(v4f& acc, float a, float b) {
  asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ float fma1(float w, float x, float acc) {
  float a;
  asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(a) : "s"(w), "v"(x), "v"(acc));
  return a;
}

template <int NV, int NM, int MT, int NU>
__global__ __launch_bounds__(256) void k_mix(float* out, const float* __restrict__ w, int iters,
                                             unsigned long long* cyc) {
  f2 a[8];
  float u[16];
  v4f m4[4];
  v4f m16[4];
  const float xv = threadIdx.x * 1e-3f;
  const f2 x = {xv, xv + 0.5f};
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = x + (float)i;
#pragma unroll
  for (int i = 0; i < 16; ++i) u[i] = xv + i;
#pragma unroll
  for (int i = 0; i < 4; ++i) m4[i] = (v4f){xv, xv + 1, xv, xv}, m16[i] = (v4f){xv, xv, xv + 2, xv};
  const f2 ws = {w[0], w[1]};
  const float ws1 = w[2];
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    // interleave: after every NV/NM VALU instructions one MFMA
    constexpr int per = NM > 0 ? (NV + NM - 1) / NM : NV;
#pragma unroll
    for (int i = 0; i < (NV > NU ? NV : NU); ++i) {
      if constexpr (NM > 0) {
        if (i % (per > 0 ? per : 1) == 0 && i / (per > 0 ? per : 1) < NM) {
          const int j = (i / (per > 0 ? per : 1)) & 3;
          if constexpr (MT == 0) mfma4(m4[j], xv, xv);
          else mfma16(m16[j], xv, xv);
        }
      }
      if (i < NV) a[i & 7] = pkfma(ws, x, a[i & 7]);
      if (i < NU) u[i & 15] = fma1(ws1, xv, u[i & 15]);
    }
    if constexpr (NV == 0 && NU == 0) {
#pragma unroll
      for (int j = 0; j < NM; ++j) {
        if constexpr (MT == 0) mfma4(m4[j & 3], xv, xv);
        else mfma16(m16[j & 3], xv, xv);
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float r = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r += a[i].x + a[i].y;
#pragma unroll
  for (int i = 0; i < 16; ++i) r += u[i];
#pragma unroll
  for (int i = 0; i < 4; ++i) r += m4[i][0] + m16[i][1];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// half the blocks (alternating) run NV pk_fma only, the other half NM MFMAs
// only: the two pipes fed by DIFFERENT waves of one SIMD
template <int NV, int NM, int MT>
__global__ __launch_bounds__(256) void k_split(float* out, const float* __restrict__ w, int iters,
                                               unsigned long long* cyc) {
  f2 a[8];
  v4f m[4];
  const float xv = threadIdx.x * 1e-3f;
  const f2 x = {xv, xv + 0.5f};
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = x + (float)i;
#pragma unroll
  for (int i = 0; i < 4; ++i) m[i] = (v4f){xv, xv + 1, xv, xv};
  const f2 ws = {w[0], w[1]};
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (blockIdx.x & 1) {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int j = 0; j < NM; ++j) {
        if constexpr (MT == 0) mfma4(m[j & 3], xv, xv);
        else mfma16(m[j & 3], xv, xv);
      }
    }
  } else {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < NV; ++i) a[i & 7] = pkfma(ws, x, a[i & 7]);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float r = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r += a[i].x + a[i].y;
#pragma unroll
  for (int i = 0; i < 4; ++i) r += m[i][0];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <class K>
void run_k(K k, const char* name, int W, int NV, int NU, int NM, int MT, float* out,
           const float* w, unsigned long long* cyc) {
  const int cus = 256, iters = 2048;
  const int blocks = cus * W;
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, w, iters, cyc);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, w, iters, cyc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> c(blocks);
  hipMemcpy(c.data(), cyc, blocks * 8, hipMemcpyDeviceToHost);
  std::sort(c.begin(), c.end());
  const double med = (double)c[blocks / 2];
  // per SIMD: W waves ran concurrently for ~med cycles
  const double cyc_it = med / iters;
  const int mcyc = MT == 0 ? 8 : 32;
  const double valu_ideal = W * (NV * 4.0 + NU * 2.0), mfma_ideal = W * NM * (double)mcyc;
  printf("{\"k\": \"%s\", \"W\": %d, \"NV_pk\": %d, \"NU\": %d, \"NM\": %d, \"mfma\": \"%s\", "
         "\"cyc_per_iter_simd\": %.1f, \"valu_ideal\": %.0f, \"mfma_ideal\": %.0f, \"ms\": %.3f, "
         "\"ghz_est\": %.3f}\n",
         name, W, NV, NU, NM, MT == 0 ? "4x4x1_16b" : "16x16x4", cyc_it, valu_ideal, mfma_ideal,
         ms, med / (ms * 1e6));
}

template <int NV, int NM, int MT, int NU>
void run(const char* name, int W, float* out, const float* w, unsigned long long* cyc) {
  run_k(k_mix<NV, NM, MT, NU>, name, W, NV, NU, NM, MT, out, w, cyc);
}

int main() {
  float* out;
  float* w;
  unsigned long long* cyc;
  hipMalloc(&out, 256 * 8 * 256 * sizeof(float));
  hipMalloc(&w, 64 * sizeof(float));
  hipMalloc(&cyc, 256 * 8 * 8);
  hipMemset(w, 0, 64 * sizeof(float));
  for (int W : {1, 2, 4, 6}) {
    run<16, 0, 0, 0>("pk_only", W, out, w, cyc);
    run<0, 0, 0, 32>("fma_only", W, out, w, cyc);
    run<0, 4, 0, 0>("mfma4_only", W, out, w, cyc);
    run<0, 4, 1, 0>("mfma16_only", W, out, w, cyc);
    run<16, 2, 0, 0>("pk16+m4x2", W, out, w, cyc);
    run<16, 4, 0, 0>("pk16+m4x4", W, out, w, cyc);
    run<16, 8, 0, 0>("pk16+m4x8", W, out, w, cyc);
    run<16, 1, 1, 0>("pk16+m16x1", W, out, w, cyc);
    run<16, 2, 1, 0>("pk16+m16x2", W, out, w, cyc);
    run<0, 4, 0, 32>("fma32+m4x4", W, out, w, cyc);
    if (W % 2 == 0) {
      // per SIMD W/2 VALU waves + W/2 MFMA waves: ideal columns are per wave
      run_k(k_split<16, 8, 0>, "split_pk16|m4x8", W, 16, 0, 8, 0, out, w, cyc);
      run_k(k_split<16, 2, 1>, "split_pk16|m16x2", W, 16, 0, 2, 1, out, w, cyc);
    }
  }
  return 0;
}
