// Launch-floor micro-benchmark for the headline k_sgpr call (VERDICT r5,
// "do this" 1): what a back-to-back launch of an EMPTY grid costs as a
// function of the grid (blocks, waves per block), its dynamic LDS allocation
// and its VGPR count; what the one-block follow-up launch (the NLL sum) adds;
// and what a kernel boundary costs behind a streaming store kernel by the
// stores' cache policy (dirty lines left in the XCD L2s at kernel end are
// written back before the next kernel may start).
// Build: hipcc -O3 --offload-arch=gfx950 -o launch_floor launch_floor.hip
// Output: one JSON line per measurement.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

// VG: 0 = whatever the body needs, 1 = forced to >= 80 VGPRs, 2 = >= 128
template <int VG>
__global__ __launch_bounds__(256) void k_empty(const float* __restrict__ in, long long B,
                                               float* out) {
  if constexpr (VG == 1) asm volatile("v_mov_b32 v79, 0" ::: "v79");
  if constexpr (VG == 2) asm volatile("v_mov_b32 v127, 0" ::: "v127");
  if (B > 0) return;
  out[threadIdx.x] = in[threadIdx.x];
}
template <int VG>
__global__ __launch_bounds__(1024) void k_empty1k(const float* __restrict__ in, long long B,
                                                  float* out) {
  if constexpr (VG == 1) asm volatile("v_mov_b32 v79, 0" ::: "v79");
  if (B > 0) return;
  out[threadIdx.x] = in[threadIdx.x];
}
template <int VG>
__global__ __launch_bounds__(512) void k_empty512(const float* __restrict__ in, long long B,
                                                  float* out) {
  if constexpr (VG == 1) asm volatile("v_mov_b32 v79, 0" ::: "v79");
  if (B > 0) return;
  out[threadIdx.x] = in[threadIdx.x];
}

// the follow-up launch's shape: one 256-thread block sums nblk 16-B records
__global__ __launch_bounds__(256) void k_tiny(const float4* __restrict__ part, int nblk,
                                              float* __restrict__ out) {
  float s = 0.f;
  for (int b = threadIdx.x; b < nblk; b += 256) s += part[b].x;
  for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off);
  __shared__ float r[4];
  if ((threadIdx.x & 63) == 0) r[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = r[0] + r[1] + r[2] + r[3];
}

// Streaming stores: every lane writes 16-B words, each wave-instruction one
// contiguous KiB, grid-stride over n4 words.  AUX: the buffer store's cache
// policy (gfx950: 1 sc0, 2 nt, 16 sc1).  LOAD: also read a same-sized input
// (nt), as k_sgpr's pass does (no compute).
template <int AUX, bool LOAD>
__global__ __launch_bounds__(256) void k_stream(const float* __restrict__ in, float* out,
                                                long long n4) {
  const auto ro = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7fffffff, 0x00020000);
  const long long stride = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
    __attribute__((ext_vector_type(4))) int v = {(int)i, 1, 2, 3};
    if constexpr (LOAD) {
      using v4i = __attribute__((ext_vector_type(4))) int;
      v = __builtin_nontemporal_load(reinterpret_cast<const v4i*>(in) + i);
    }
    // offsets past 2 GB do not occur here (buffers below 128 MB)
    __builtin_amdgcn_raw_buffer_store_b128(v, ro, (int)(i * 16), 0, AUX);
  }
}

static float time_launches(hipStream_t st, int n, auto&& launch) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 20; ++i) launch(i);
  CK(hipStreamSynchronize(st));
  CK(hipEventRecord(e0, st));
  for (int i = 0; i < n; ++i) launch(i);
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return ms * 1e3f / n;  // us per launch
}

int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 2000;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  float *in, *out, *part, *red;
  CK(hipMalloc(&in, 1 << 20));
  CK(hipMalloc(&out, 1 << 20));
  CK(hipMalloc(&part, 6144 * 16));
  CK(hipMalloc(&red, 64));
  CK(hipMemset(part, 0, 6144 * 16));
  const long long B = 1 << 20;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  // 1. empty 256-thread grids: blocks x LDS x VGPRs, alone and with the follow-up
  const int grids[] = {256, 512, 768, 1024, 1536, 2048};
  const size_t ldss[] = {0, 20480};
  for (int vg = 0; vg < 3; ++vg)
    for (size_t lds : ldss)
      for (int g : grids) {
        auto one = [&](int) {
          if (vg == 0) hipLaunchKernelGGL(k_empty<0>, dim3(g), dim3(256), lds, st, in, B, out);
          if (vg == 1) hipLaunchKernelGGL(k_empty<1>, dim3(g), dim3(256), lds, st, in, B, out);
          if (vg == 2) hipLaunchKernelGGL(k_empty<2>, dim3(g), dim3(256), lds, st, in, B, out);
        };
        const float t1 = time_launches(st, N, one);
        const float t2 = time_launches(st, N, [&](int i) {
          one(i);
          hipLaunchKernelGGL(k_tiny, dim3(1), dim3(256), 0, st, (const float4*)part, g, red);
        });
        printf("{\"test\": \"empty\", \"block\": 256, \"blocks\": %d, \"lds\": %zu, \"vgpr\": \"%s\", "
               "\"us\": %.3f, \"with_followup_us\": %.3f}\n",
               g, lds, vg == 0 ? "min" : (vg == 1 ? ">=80" : ">=128"), t1, t2);
        fflush(stdout);
      }
  // 2. the same waves in bigger blocks (1536 x 4 waves = 768 x 8 = 384 x 16)
  for (int vg = 0; vg < 2; ++vg) {
    const float a = time_launches(st, N, [&](int) {
      if (vg) hipLaunchKernelGGL(k_empty512<1>, dim3(768), dim3(512), 40960, st, in, B, out);
      else hipLaunchKernelGGL(k_empty512<0>, dim3(768), dim3(512), 40960, st, in, B, out);
    });
    const float b = time_launches(st, N, [&](int) {
      if (vg) hipLaunchKernelGGL(k_empty1k<1>, dim3(384), dim3(1024), 81920, st, in, B, out);
      else hipLaunchKernelGGL(k_empty1k<0>, dim3(384), dim3(1024), 81920, st, in, B, out);
    });
    printf("{\"test\": \"empty_big_blocks\", \"vgpr\": \"%s\", \"768x512_us\": %.3f, "
           "\"384x1024_us\": %.3f}\n", vg ? ">=80" : "min", a, b);
    fflush(stdout);
  }
  // 3. boundary behind streaming stores: 44 MB (k_sgpr's z at 2^20 rows) and
  //    88 MB, over rotating buffers (>= 1 GB in all), by cache policy
  const long long zbytes[] = {44040192LL, 88080384LL};
  const int nrot = 12;
  std::vector<float*> bufs(nrot), ins(nrot);
  for (int i = 0; i < nrot; ++i) {
    CK(hipMalloc(&bufs[i], 88080384LL));
    CK(hipMalloc(&ins[i], 88080384LL));
    CK(hipMemset(ins[i], 0, 88080384LL));
  }
  const int grid = 6 * cus;
  struct Pol {
    const char* name;
    int aux;
  } pols[] = {{"plain", 0}, {"nt", 2}, {"sc1", 16}, {"sc0sc1", 17}, {"sc1nt", 18}, {"sc0sc1nt", 19}};
  for (long long zb : zbytes)
    for (int ld = 0; ld < 2; ++ld)
      for (const Pol& p : pols) {
        const long long n4 = zb / 16;
        auto one = [&](int i) {
          float* o = bufs[i % nrot];
          const float* x = ins[(i + 5) % nrot];
#define CNF_LF_CASE(A)                                                                        \
  if (p.aux == A) {                                                                           \
    if (ld) hipLaunchKernelGGL((k_stream<A, true>), dim3(grid), dim3(256), 0, st, x, o, n4);  \
    else hipLaunchKernelGGL((k_stream<A, false>), dim3(grid), dim3(256), 0, st, x, o, n4);    \
  }
          CNF_LF_CASE(0) CNF_LF_CASE(2) CNF_LF_CASE(16) CNF_LF_CASE(17) CNF_LF_CASE(18)
          CNF_LF_CASE(19)
#undef CNF_LF_CASE
        };
        const float t1 = time_launches(st, N / 4, one);
        const float t2 = time_launches(st, N / 4, [&](int i) {
          one(i);
          hipLaunchKernelGGL(k_tiny, dim3(1), dim3(256), 0, st, (const float4*)part, grid, red);
        });
        const double bytes = (double)zb * (ld ? 2 : 1);
        printf("{\"test\": \"stream\", \"policy\": \"%s\", \"load\": %d, \"store_MB\": %.1f, "
               "\"blocks\": %d, \"us\": %.3f, \"TBps\": %.3f, \"with_followup_us\": %.3f}\n",
               p.name, ld, zb / 1048576.0, grid, t1, bytes / (t1 * 1e-6) / 1e12, t2);
        fflush(stdout);
      }
  return 0;
}
