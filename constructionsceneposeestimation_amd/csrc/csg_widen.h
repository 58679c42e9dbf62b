// Host side of the narrowed instance-id wire (csg_api.cpp, host-output
// batches).  The reference hands its caller an int32 instance mask
// (generate_construction_data.py:1909-1910, the .npy of :2066-2069); with at
// most 255 labels an id fits one byte as (id + 1), so the device writes the
// ids as 1- (or 2-) byte values (k_narrow_ids), a quarter of the int32 bytes
// cross PCIe, and this pool of host threads widens them into the caller's
// int32 array: dst[i] = src[i] - 1.  A launch chain's ids are widened while
// later chains render and copy; the batch's stream waits for the widening
// (WidenLatch::wait in a host function on the copy stream), so "the stream
// is done" still means "the int32 ids are in place".
#pragma once
#include <immintrin.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace csg {

// Outstanding widening tasks of one batch.
struct WidenLatch {
  std::mutex m;
  std::condition_variable cv;
  size_t pending = 0;
  void add(size_t k) {
    std::lock_guard<std::mutex> g(m);
    pending += k;
  }
  void done() {
    std::lock_guard<std::mutex> g(m);
    if (--pending == 0) cv.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> g(m);
    cv.wait(g, [&] { return pending == 0; });
  }
};

// dst[i] = (int32)src[i] - 1 for 1- or 2-byte sources.  AVX2 when the CPU has
// it: zero-extend 8 ids per 256-bit lane group, subtract 1, stream the int32s
// past the caches (the caller reads them much later, from a writer thread).
__attribute__((target("avx2"))) inline void widen_avx2(const void* src, uint32_t bytes, int32_t* dst, size_t n) {
  size_t i = 0;
  const uint8_t* s8 = static_cast<const uint8_t*>(src);
  const uint16_t* s16 = static_cast<const uint16_t*>(src);
  auto one = [&](size_t k) { dst[k] = (bytes == 1 ? (int32_t)s8[k] : (int32_t)s16[k]) - 1; };
  for (; i < n && ((uintptr_t)(dst + i) & 31u); ++i) one(i);
  const __m256i m1 = _mm256_set1_epi32(1);
  if (bytes == 1) {
    for (; i + 32 <= n; i += 32) {
      const __m128i lo = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s8 + i));
      const __m128i hi = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s8 + i + 16));
      _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i), _mm256_sub_epi32(_mm256_cvtepu8_epi32(lo), m1));
      _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 8),
                          _mm256_sub_epi32(_mm256_cvtepu8_epi32(_mm_srli_si128(lo, 8)), m1));
      _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 16), _mm256_sub_epi32(_mm256_cvtepu8_epi32(hi), m1));
      _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 24),
                          _mm256_sub_epi32(_mm256_cvtepu8_epi32(_mm_srli_si128(hi, 8)), m1));
    }
  } else {
    for (; i + 16 <= n; i += 16) {
      const __m128i lo = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s16 + i));
      const __m128i hi = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s16 + i + 8));
      _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i), _mm256_sub_epi32(_mm256_cvtepu16_epi32(lo), m1));
      _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 8), _mm256_sub_epi32(_mm256_cvtepu16_epi32(hi), m1));
    }
  }
  for (; i < n; ++i) one(i);
  _mm_sfence();
}

inline void widen_ids(const void* src, uint32_t bytes, int32_t* dst, size_t n) {
  static const bool avx2 = __builtin_cpu_supports("avx2");
  if (avx2) {
    widen_avx2(src, bytes, dst, n);
    return;
  }
  const uint8_t* s8 = static_cast<const uint8_t*>(src);
  const uint16_t* s16 = static_cast<const uint16_t*>(src);
  for (size_t i = 0; i < n; ++i) dst[i] = (bytes == 1 ? (int32_t)s8[i] : (int32_t)s16[i]) - 1;
}

// Process-wide pool of widening threads (CSG_WIDEN_THREADS, default the
// process's CPU share: OMP_NUM_THREADS when set -- the GPU box sets it to its
// 16-CPU share -- else the hardware threads, at most 16).  Never destroyed:
// HIP host functions of a context being torn down at exit may still submit.
class WidenPool {
 public:
  struct Task {
    const void* src;
    uint32_t bytes;
    int32_t* dst;
    size_t n;
    std::shared_ptr<WidenLatch> latch;
  };
  static WidenPool& get() {
    static WidenPool* p = new WidenPool();
    return *p;
  }
  static unsigned default_threads() {
    unsigned t = 0;
    if (const char* v = getenv("CSG_WIDEN_THREADS")) t = (unsigned)atoi(v);
    if (!t) {
      if (const char* v = getenv("OMP_NUM_THREADS")) t = (unsigned)atoi(v);
      if (!t) t = std::max(1u, std::thread::hardware_concurrency());
      t = std::min(t, 16u);
    }
    return std::max(1u, std::min(t, 256u));
  }
  // Split [0, n) into pieces of ~kPiece ids (whole 64-id groups) and queue them.
  void submit(const void* src, uint32_t bytes, int32_t* dst, size_t n, const std::shared_ptr<WidenLatch>& latch) {
    constexpr size_t kPiece = 1u << 20;
    const size_t pieces = std::max<size_t>(1, (n + kPiece - 1) / kPiece);
    latch->add(pieces);
    {
      std::lock_guard<std::mutex> g(m_);
      for (size_t k = 0; k < pieces; ++k) {
        const size_t a = k * kPiece, b = std::min(n, a + kPiece);
        q_.push_back(Task{static_cast<const uint8_t*>(src) + a * bytes, bytes, dst + a, b - a, latch});
      }
    }
    cv_.notify_all();
  }

 private:
  WidenPool() {
    const unsigned t = default_threads();
    for (unsigned k = 0; k < t; ++k) std::thread([this] { run(); }).detach();
  }
  void run() {
    for (;;) {
      Task t;
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return !q_.empty(); });
        t = q_.front();
        q_.pop_front();
      }
      widen_ids(t.src, t.bytes, t.dst, t.n);
      t.latch->done();
    }
  }
  std::mutex m_;
  std::condition_variable cv_;
  std::deque<Task> q_;
};

}  // namespace csg
