"""CPU tests of csg_deflate.h, the sequential pieces of the GPU file encoders
(csg_encode.hip): a one-thread harness (tests/deflate_host.cpp) built from the
same helpers writes PNGs that zlib must decode to the input pixels (CRCs and
Adler-32 checked), "%.6f" text byte-identical to np.savetxt, and
length-limited Huffman codes that are complete and optimal when the limit
does not bind."""
import heapq
import io
import os
import subprocess

import numpy as np
import pytest

from pngutil import decode_png

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    d = tmp_path_factory.mktemp("deflate")
    exe = str(d / "deflate_host")
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", os.path.join(HERE, "deflate_host.cpp"), "-o", exe],
                   check=True)
    return exe, d


def _images(rng=np.random.default_rng(7)):
    flat = np.full((9, 400, 3), 37, np.uint8)                       # runs far longer than 258
    grad = np.broadcast_to(np.arange(300, dtype=np.uint8)[None, :, None], (5, 300, 3)).copy()
    noise = rng.integers(0, 256, (13, 29, 3), dtype=np.uint8)        # incompressible
    blocks = np.repeat(np.repeat(rng.integers(0, 256, (4, 6, 3), dtype=np.uint8), 5, 0), 7, 1)
    ones = np.ones((3, 11, 3), np.uint8)                             # runs that include the filter byte
    return [np.zeros((1, 1, 3), np.uint8), rng.integers(0, 256, (2, 3, 3), dtype=np.uint8), flat, grad, noise,
            blocks, ones]


@pytest.mark.parametrize("k", range(7))
def test_png_roundtrip(harness, k):
    exe, d = harness
    img = _images()[k]
    H, W, _ = img.shape
    src, dst = str(d / f"i{k}.rgb"), str(d / f"o{k}.png")
    img.tofile(src)
    subprocess.run([exe, "png", str(W), str(H), src, dst], check=True)
    assert np.array_equal(decode_png(open(dst, "rb").read()), img)


def test_csv_matches_savetxt(harness):
    exe, d = harness
    specials = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-7, 5e-7, 4.9999997e-7, 2.0 ** -21, 0.5, 1.0,
                         2.0 ** 40, 2.0 ** 41, 3.4028235e38, -3.4028235e38, 1e20, 1.4e-45, 123.456789,
                         0.0000005, 0.0000015, 0.0000025, 249.99998, 0.5000001, 7.0e15, 16777217.0],
                        np.float32)
    rng = np.random.default_rng(3)
    rand = np.concatenate([rng.uniform(0.5, 250.0, 200), rng.uniform(-1e6, 1e6, 50),
                           rng.standard_normal(50) * 1e-6]).astype(np.float32)
    vals = np.concatenate([specials, rand, np.zeros(300 - specials.size - rand.size + 25, np.float32)])[:300]
    img = vals.reshape(12, 25)
    src, dst = str(d / "v.f32"), str(d / "v.csv")
    img.tofile(src)
    subprocess.run([exe, "csv", "25", "12", src, dst], check=True)
    ref = io.BytesIO()
    np.savetxt(ref, img, fmt="%.6f", delimiter=" ")
    assert open(dst, "rb").read() == ref.getvalue()


def huffman_cost(freq):
    h = [(f, i) for i, f in enumerate(freq) if f]
    if len(h) < 2:
        return sum(freq)
    heapq.heapify(h)
    cost, n = 0, len(freq)
    while len(h) > 1:
        a, b = heapq.heappop(h), heapq.heappop(h)
        cost += a[0] + b[0]
        heapq.heappush(h, (a[0] + b[0], n))
        n += 1
    return cost


@pytest.mark.parametrize("case", ["random", "fibonacci", "skewed", "two", "one", "flat"])
def test_huffman_lengths(harness, case):
    exe, _ = harness
    rng = np.random.default_rng(11)
    if case == "random":
        freq = list(rng.integers(0, 1000, 286) * (rng.random(286) < 0.7))
    elif case == "fibonacci":        # optimal code needs lengths far beyond 15
        fib = [1, 1]
        while len(fib) < 40:
            fib.append(fib[-1] + fib[-2])
        freq = fib + [0] * 10
    elif case == "skewed":
        freq = [10 ** 6] + [1] * 285
    elif case == "two":
        freq = [0, 5, 0, 9]
    elif case == "one":
        freq = [0, 0, 7, 0]
    else:
        freq = [3] * 19
    for maxbits in (15, 7):
        out = subprocess.run([exe, "huff", str(maxbits)] + [str(int(f)) for f in freq], check=True,
                             capture_output=True, text=True).stdout
        lens = [int(x) for x in out.split()]
        used = [i for i, f in enumerate(freq) if f]
        assert all(lens[i] == 0 for i in range(len(freq)) if not freq[i])
        if len(used) == 1:
            assert lens[used[0]] == 1
            continue
        if len(used) > 2 ** maxbits:
            continue
        assert max(lens) <= maxbits
        assert sum(2.0 ** -lens[i] for i in used) == 1.0           # complete prefix code
        cost = sum(freq[i] * lens[i] for i in used)
        opt = huffman_cost(freq)
        assert cost >= opt
        if case in ("random", "two", "flat") and maxbits == 15:
            assert cost == opt
