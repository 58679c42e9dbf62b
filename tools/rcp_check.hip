// Exhaustive check, on the GPU, that a short reciprocal equals the IEEE
// division 1.0f / x bit for bit over a range of x.
//
//   fast(x): r0 = v_rcp_f32(x) (hardware approximation, ~1 ulp);
//            e  = fma(-x, r0, 1)   (the residual, exact in one rounding);
//            r  = fma(e, r0, r0)   (one Newton step)
//   ieee(x): 1.0f / x as hipcc compiles it under -ffp-contract=off (the
//            v_div_scale / v_div_fmas / v_div_fixup sequence the kernels use)
//
// Every float bit pattern in [lo, hi) is tested (all positive normals by
// default: 2^31 - 2^23 - ... patterns); the program prints one JSON line with
// the number tested, the mismatches and the first few of them.
//   hipcc -O3 -ffp-contract=off --offload-arch=gfx950 -o rcp_check tools/rcp_check.hip
//   ./rcp_check [lo_bits hi_bits]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ float fast_rcp(float x) {
  const float r0 = __builtin_amdgcn_rcpf(x);
  const float e = __builtin_fmaf(-x, r0, 1.0f);
  return __builtin_fmaf(e, r0, r0);
}

__global__ void k_check(uint32_t lo, uint64_t n, unsigned long long* bad, uint32_t* first, uint32_t* nfirst) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint32_t bits = lo + (uint32_t)i;
    const float x = __uint_as_float(bits);
    const float a = fast_rcp(x);
    const float b = 1.0f / x;
    if (__float_as_uint(a) != __float_as_uint(b)) {
      atomicAdd(bad, 1ull);
      const uint32_t k = atomicAdd(nfirst, 1u);
      if (k < 16) first[k] = bits;
    }
  }
}

int main(int argc, char** argv) {
  uint32_t lo = 0x00800000u, hi = 0x7F800000u;   // smallest normal .. +inf (excluded)
  if (argc >= 3) {
    lo = (uint32_t)strtoul(argv[1], nullptr, 0);
    hi = (uint32_t)strtoul(argv[2], nullptr, 0);
  }
  const uint64_t n = (uint64_t)(hi - lo);
  unsigned long long* d_bad;
  uint32_t *d_first, *d_nfirst;
  if (hipMalloc(&d_bad, 8) != hipSuccess || hipMalloc(&d_first, 64) != hipSuccess ||
      hipMalloc(&d_nfirst, 4) != hipSuccess) {
    fprintf(stderr, "hipMalloc failed\n");
    return 1;
  }
  (void)hipMemset(d_bad, 0, 8);
  (void)hipMemset(d_nfirst, 0, 4);
  hipLaunchKernelGGL(k_check, dim3(4096), dim3(256), 0, 0, lo, n, d_bad, d_first, d_nfirst);
  if (hipDeviceSynchronize() != hipSuccess) {
    fprintf(stderr, "kernel failed\n");
    return 1;
  }
  unsigned long long bad = 0;
  uint32_t first[16] = {}, nfirst = 0;
  (void)hipMemcpy(&bad, d_bad, 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(first, d_first, 64, hipMemcpyDeviceToHost);
  (void)hipMemcpy(&nfirst, d_nfirst, 4, hipMemcpyDeviceToHost);
  printf("{\"lo\": \"0x%08x\", \"hi\": \"0x%08x\", \"tested\": %llu, \"mismatches\": %llu, \"first\": [", lo, hi,
         (unsigned long long)n, bad);
  for (uint32_t k = 0; k < nfirst && k < 16; ++k) printf("%s\"0x%08x\"", k ? ", " : "", first[k]);
  printf("]}\n");
  return 0;
}
