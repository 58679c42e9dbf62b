// SQ counter calibration on gfx950 (VERDICT r05 "next" 1a): what the VALU,
// wait and wave-cycle counters read for kernels of known behaviour, so the
// k_raster / k_setup "busy" figures rest on a measured scale instead of a
// formula.  Each kernel runs a known number of wave64 VALU instructions:
//   k_fma_indep<W>  8 independent v_fma_f32 chains per lane, W waves per SIMD
//                   (grid 256 CUs x W workgroups of 4 waves): the issue-bound case
//   k_fma_dep<W>    one dependent v_fma_f32 chain per lane (latency-bound issue)
//   k_barrier       wave 0 of each 4-wave workgroup runs a dependent chain, the
//                   other three wait at s_barrier: where barrier parking lands
//   k_lds_chain     dependent ds_read_b32 pointer chase: lgkmcnt parking
//   k_mem_chain     dependent global_load_dword pointer chase over 1 GiB: vmcnt parking
// Timed with HIP events; tools/calib_valu.sh runs the counter passes and
// tools/calib_valu_summary.py relates counters to instructions and cycles.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr int kIter = 65536;   // loop trips; each trip issues 8 v_fma_f32 per wave

#define FMA(a) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a) : "v"(x), "v"(y))

template <int W>
__global__ __launch_bounds__(256) void k_fma_indep(float* out, float x, float y, int iters) {
  float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int i = 0; i < iters; ++i) {
    FMA(a0); FMA(a1); FMA(a2); FMA(a3); FMA(a4); FMA(a5); FMA(a6); FMA(a7);
  }
  out[blockIdx.x * 256 + threadIdx.x] = ((a0 + a1) + (a2 + a3)) + ((a4 + a5) + (a6 + a7));
}

template <int W>
__global__ __launch_bounds__(256) void k_fma_dep(float* out, float x, float y, int iters) {
  float a0 = threadIdx.x;
  for (int i = 0; i < iters; ++i) {
    FMA(a0); FMA(a0); FMA(a0); FMA(a0); FMA(a0); FMA(a0); FMA(a0); FMA(a0);
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0;
}

// wave 0 works (8 dependent FMAs per trip, `inner` trips), waves 1-3 park at
// the barrier; `outer` barriers per workgroup
__global__ __launch_bounds__(256) void k_barrier(float* out, float x, float y, int outer, int inner) {
  float a0 = threadIdx.x;
  for (int o = 0; o < outer; ++o) {
    if (threadIdx.x < 64) {
      for (int i = 0; i < inner; ++i) { FMA(a0); FMA(a0); FMA(a0); FMA(a0); FMA(a0); FMA(a0); FMA(a0); FMA(a0); }
    }
    __syncthreads();
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0;
}

__global__ __launch_bounds__(256) void k_lds_chain(uint32_t* out, int iters) {
  __shared__ uint32_t nxt[4096];
  for (int i = threadIdx.x; i < 4096; i += 256) nxt[i] = (uint32_t)((i * 1031 + 7) & 4095);
  __syncthreads();
  uint32_t p = threadIdx.x;
  for (int i = 0; i < iters; ++i) p = nxt[p];
  out[blockIdx.x * 256 + threadIdx.x] = p;
}

__global__ __launch_bounds__(256) void k_mem_chain(const uint32_t* __restrict__ nxt, uint32_t* out, int iters) {
  uint32_t p = (blockIdx.x * 256 + threadIdx.x) * 977u;
  for (int i = 0; i < iters; ++i) p = nxt[p & ((1u << 28) - 1u)];
  out[blockIdx.x * 256 + threadIdx.x] = p;
}

struct Timer {
  hipEvent_t a, b;
  Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
  float ms() { float m; CK(hipEventElapsedTime(&m, a, b)); return m; }
};

int main() {
  hipDeviceProp_t pr;
  CK(hipGetDeviceProperties(&pr, 0));
  const int cus = pr.multiProcessorCount;
  float* fo;
  uint32_t *uo, *chain;
  CK(hipMalloc(&fo, (size_t)cus * 16 * 256 * 4));
  CK(hipMalloc(&uo, (size_t)cus * 16 * 256 * 4));
  const size_t n_chain = 1ull << 28;   // 1 GiB of u32
  CK(hipMalloc(&chain, n_chain * 4));
  {
    std::vector<uint32_t> h(1u << 20);
    for (size_t base = 0; base < n_chain; base += h.size()) {
      for (size_t i = 0; i < h.size(); ++i) h[i] = (uint32_t)(((base + i) * 2654435761ull + 12345u) & (n_chain - 1));
      CK(hipMemcpy(chain + base, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    }
  }
  Timer t;
  printf("{\"cus\": %d, \"clock_khz\": %d, \"iter\": %d, \"kernels\": [", cus, pr.clockRate, kIter);
  bool first = true;
  auto rec = [&](const char* name, int blocks, double valu_per_wave, double extra) {
    const float ms = t.ms();
    printf("%s{\"name\": \"%s\", \"blocks\": %d, \"waves\": %d, \"valu_per_wave\": %.0f, \"ms\": %.4f, \"x\": %.0f}",
           first ? "" : ", ", name, blocks, blocks * 4, valu_per_wave, ms, extra);
    first = false;
  };
  // warm-up
  hipLaunchKernelGGL(k_fma_indep<1>, dim3(cus), dim3(256), 0, 0, fo, 1.0f, 0.5f, 64);
  CK(hipDeviceSynchronize());
  // VALU body: 8 FMAs per trip (+ the epilogue's 7 adds, the 8 initial converts and adds: counted below)
  const double body = 8.0 * kIter;
#define RUN_INDEP(W)                                                                              \
  CK(hipEventRecord(t.a));                                                                        \
  hipLaunchKernelGGL(k_fma_indep<W>, dim3(cus * W), dim3(256), 0, 0, fo, 1.0f, 0.5f, kIter);      \
  CK(hipEventRecord(t.b));                                                                        \
  CK(hipEventSynchronize(t.b));                                                                   \
  rec("k_fma_indep<" #W ">", cus * W, body, W);
  RUN_INDEP(1) RUN_INDEP(2) RUN_INDEP(4) RUN_INDEP(8)
#define RUN_DEP(W)                                                                                \
  CK(hipEventRecord(t.a));                                                                        \
  hipLaunchKernelGGL(k_fma_dep<W>, dim3(cus * W), dim3(256), 0, 0, fo, 1.0f, 0.5f, kIter);        \
  CK(hipEventRecord(t.b));                                                                        \
  CK(hipEventSynchronize(t.b));                                                                   \
  rec("k_fma_dep<" #W ">", cus * W, body, W);
  RUN_DEP(1) RUN_DEP(8)
  // barrier: 2 workgroups per CU (2 waves per SIMD), wave 0 runs 64 FMAs per barrier
  CK(hipEventRecord(t.a));
  hipLaunchKernelGGL(k_barrier, dim3(cus * 2), dim3(256), 0, 0, fo, 1.0f, 0.5f, 8192, 8);
  CK(hipEventRecord(t.b));
  CK(hipEventSynchronize(t.b));
  rec("k_barrier", cus * 2, 8192.0 * 64.0 / 4.0, 8192);   // x: barriers per workgroup; VALU averaged over the 4 waves
  CK(hipEventRecord(t.a));
  hipLaunchKernelGGL(k_lds_chain, dim3(cus * 2), dim3(256), 0, 0, uo, 65536);
  CK(hipEventRecord(t.b));
  CK(hipEventSynchronize(t.b));
  rec("k_lds_chain", cus * 2, 0, 65536);
  CK(hipEventRecord(t.a));
  hipLaunchKernelGGL(k_mem_chain, dim3(cus * 2), dim3(256), 0, 0, chain, uo, 1024);
  CK(hipEventRecord(t.b));
  CK(hipEventSynchronize(t.b));
  rec("k_mem_chain", cus * 2, 0, 1024);
  printf("]}\n");
  CK(hipFree(fo));
  CK(hipFree(uo));
  CK(hipFree(chain));
  return 0;
}
