"""The host side of the narrowed instance-id wire (csrc/csg_widen.h), on the
CPU: the widening dst[i] = src[i] - 1 of 1- and 2-byte ids into int32, by the
AVX2 path and the scalar one, for every tail length and destination
alignment, and through the WidenPool threads and their latch -- against
numpy.  The reference's mask is int32 with -1 background
(generate_construction_data.py:1909-1910); the wire carries id + 1.

The header is compiled here with g++ into a small test library (no GPU)."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = r"""
#include "csg_widen.h"
#include <memory>
extern "C" void widen(const void* src, uint32_t bytes, int32_t* dst, size_t n) { csg::widen_ids(src, bytes, dst, n); }
extern "C" void widen_scalar(const void* src, uint32_t bytes, int32_t* dst, size_t n) {
  const uint8_t* s8 = static_cast<const uint8_t*>(src);
  const uint16_t* s16 = static_cast<const uint16_t*>(src);
  for (size_t i = 0; i < n; ++i) dst[i] = (bytes == 1 ? (int32_t)s8[i] : (int32_t)s16[i]) - 1;
}
extern "C" int has_avx2() { return __builtin_cpu_supports("avx2") ? 1 : 0; }
// k submissions of consecutive slices through the pool, then one wait
extern "C" void widen_pool(const void* src, uint32_t bytes, int32_t* dst, size_t n, size_t k) {
  auto latch = std::make_shared<csg::WidenLatch>();
  const size_t step = (n + k - 1) / k;
  for (size_t a = 0; a < n; a += step) {
    const size_t m = n - a < step ? n - a : step;
    csg::WidenPool::get().submit(static_cast<const uint8_t*>(src) + a * bytes, bytes, dst + a, m, latch);
  }
  latch->wait();
}
"""


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    d = tmp_path_factory.mktemp("widen")
    src = d / "widen_test.cpp"
    src.write_text(HARNESS)
    so = d / "libwiden_test.so"
    inc = os.path.join(ROOT, "constructionsceneposeestimation_amd", "csrc")
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-pthread", "-I", inc, str(src), "-o", str(so)],
                   check=True, capture_output=True)
    lb = C.CDLL(str(so))
    for f in (lb.widen, lb.widen_scalar):
        f.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_size_t]
    lb.widen_pool.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_size_t, C.c_size_t]
    return lb


def _ids(rng, n, bytes_):
    hi = 255 if bytes_ == 1 else 65535
    return rng.integers(0, hi + 1, n).astype(np.uint8 if bytes_ == 1 else np.uint16)


@pytest.mark.parametrize("bytes_", [1, 2])
def test_every_tail_and_alignment(lib, bytes_):
    rng = np.random.default_rng(bytes_)
    for n in list(range(0, 80)) + [255, 256, 257, 1023, 4099]:
        src = _ids(rng, n + 3, bytes_)
        for so in range(3):                    # source offset (unaligned loads)
            s = src[so:so + n]
            want = s.astype(np.int32) - 1
            for do in range(9):                # destination offset in int32s: every 32-B alignment
                buf = np.full(n + 16, 12345, np.int32)
                lib.widen(s.ctypes.data, bytes_, buf[do:].ctypes.data, n)
                assert np.array_equal(buf[do:do + n], want), (n, so, do)
                assert (buf[:do] == 12345).all() and (buf[do + n:] == 12345).all(), (n, so, do)


@pytest.mark.parametrize("bytes_", [1, 2])
def test_full_range_matches_scalar_and_numpy(lib, bytes_):
    n = 1 << 16 if bytes_ == 1 else 1 << 17
    s = np.arange(n).astype(np.uint8 if bytes_ == 1 else np.uint16)   # every value, both ends
    a = np.empty(n, np.int32)
    b = np.empty(n, np.int32)
    lib.widen(s.ctypes.data, bytes_, a.ctypes.data, n)
    lib.widen_scalar(s.ctypes.data, bytes_, b.ctypes.data, n)
    assert np.array_equal(a, b)
    assert np.array_equal(a, s.astype(np.int32) - 1)
    assert a.min() == -1 and a.max() == (254 if bytes_ == 1 else 65534)


def test_avx2_dispatch_follows_the_cpu(lib):
    """widen_ids takes the AVX2 loop exactly when the CPU reports AVX2 (the GPU
    box's EPYC does); otherwise the scalar loop, with the same results."""
    try:
        flags = open("/proc/cpuinfo").read().split()
    except OSError:
        pytest.skip("no /proc/cpuinfo")
    assert lib.has_avx2() == (1 if "avx2" in flags else 0)


@pytest.mark.parametrize("bytes_", [1, 2])
def test_pool_pieces_and_latch(lib, bytes_):
    rng = np.random.default_rng(7 + bytes_)
    n = 3 * (1 << 20) + 4321           # several 1 M-id pieces per submission, ragged end
    s = _ids(rng, n, bytes_)
    for k in (1, 3, 7):
        out = np.full(n + 1, 777, np.int32)
        lib.widen_pool(s.ctypes.data, bytes_, out[1:].ctypes.data, n, k)
        assert np.array_equal(out[1:], s.astype(np.int32) - 1), k
        assert out[0] == 777
