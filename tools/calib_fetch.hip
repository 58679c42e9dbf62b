// FETCH_SIZE calibration for k_raster's access patterns (MI355X_MICROARCH.md
// §HBM: "calibrate on a known byte count in your own access pattern").
// Each kernel touches a known set of 128-B lines of a 2 GiB buffer (far past
// the 256 MiB Infinity Cache), once each, in random order:
//   k_gather4   one 4-B load per line (texture taps, bin ids)
//   k_rec112    one 112-B record (7 x 16-B loads) per slot, records back to back
//   k_stream16  16 B per lane, contiguous (the guide's calibrated pattern)
// Run under rocprofv3 --pmc FETCH_SIZE; tools/calib_fetch.py prints
// FETCH_SIZE * 1024 / bytes touched for each.
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

__global__ void k_gather4(const uint32_t* __restrict__ buf, const uint32_t* __restrict__ line, uint32_t* out,
                          uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = buf[(size_t)line[i] * 32u];
}

__global__ void k_rec112(const uint4* __restrict__ buf, const uint32_t* __restrict__ rec, uint4* out, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const uint4* p = buf + (size_t)rec[i] * 7u;
    uint4 a = p[0];
#pragma unroll
    for (int k = 1; k < 7; ++k) {
      const uint4 b = p[k];
      a.x ^= b.x; a.y ^= b.y; a.z ^= b.z; a.w ^= b.w;
    }
    out[i] = a;
  }
}

__global__ void k_stream16(const uint4* __restrict__ buf, uint4* out, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const uint4 a = buf[i];
    if (a.x == 0x12345678u && a.y == 0x9abcdef0u) out[0] = a;   // (never true: keeps the load, writes nothing)
  }
}

int main() {
  const size_t bytes = 2ull << 30;                  // 2 GiB
  const uint32_t n_lines = (uint32_t)(bytes / 128);
  const uint32_t n = 1u << 22;                      // 4 Mi lines / records touched (512 MiB / 448 MiB)
  uint8_t* buf;
  CK(hipMalloc(&buf, bytes));
  CK(hipMemset(buf, 1, bytes));
  // random distinct lines: a multiplicative permutation of the line index space
  std::vector<uint32_t> line(n), rec(n);
  const uint32_t n_recs = (uint32_t)(bytes / 112);
  for (uint32_t i = 0; i < n; ++i) {
    line[i] = (uint32_t)(((uint64_t)i * 2654435761ull) % n_lines);
    rec[i] = (uint32_t)(((uint64_t)i * 2246822519ull) % n_recs);
  }
  uint32_t *d_line, *d_rec;
  uint4* d_out;
  CK(hipMalloc(&d_line, n * 4));
  CK(hipMalloc(&d_rec, n * 4));
  CK(hipMalloc(&d_out, (size_t)n * 16));
  CK(hipMemcpy(d_line, line.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_rec, rec.data(), n * 4, hipMemcpyHostToDevice));
  const uint32_t n16 = (uint32_t)((size_t)n * 128 / 16);   // 512 MiB streamed
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(k_gather4, dim3((n + 255) / 256), dim3(256), 0, 0, (const uint32_t*)buf, d_line,
                       (uint32_t*)d_out, n);
    hipLaunchKernelGGL(k_rec112, dim3((n + 255) / 256), dim3(256), 0, 0, (const uint4*)buf, d_rec, d_out, n);
    hipLaunchKernelGGL(k_stream16, dim3((n16 + 255) / 256), dim3(256), 0, 0, (const uint4*)buf, d_out, n16);
  }
  CK(hipDeviceSynchronize());
  printf("{\"n\": %u, \"gather4_lines_bytes\": %llu, \"rec112_bytes\": %llu, \"stream16_bytes\": %llu, "
         "\"index_bytes\": %u}\n",
         n, (unsigned long long)n * 128ull, (unsigned long long)n * 112ull, (unsigned long long)n16 * 16ull, n * 4);
  CK(hipFree(buf));
  CK(hipFree(d_line));
  CK(hipFree(d_rec));
  CK(hipFree(d_out));
  return 0;
}
