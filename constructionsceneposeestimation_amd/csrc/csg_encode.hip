// csg_encode.hip — the generator's files encoded on the GPU from a rendered
// batch still in HBM (csg_outputs.file_kinds, include/csg_api.h): the RGB
// PNG and the JET depth PNG (cv2.imwrite, generate_construction_data.py
// :1672-1673, :1690-1709), the depth CSV (np.savetxt "%.6f" :1687-1688) and
// the point-cloud TXT (np.savetxt of x y z r g b, :766-770, :1756-1757).
// The host then only copies the packed bytes out and writes them.
//
// Work is parallel over segments of image rows (PNG: one thread per 512 raw
// bytes of a row; text: one wave per 64 pixels of a row):
//
//   PNG, per image kind (csg_deflate.h for the formats):
//     k_png_scan    Sub-filter the row on the fly, run-length tokens -> the
//                   frame's literal/length histogram (LDS, then one atomic
//                   per symbol per block), Adler-32 sums of the row
//     k_png_codes   one workgroup per frame: rank sort of the used symbols,
//                   length-limited Huffman code, canonical codes, zlib +
//                   dynamic-block header bits, Adler-32 of the frame
//     k_png_bits    the row's bit count under those codes
//     k_png_layout  one workgroup per frame: row bit offsets (block scan),
//                   stream / file size
//   Text (CSV, point cloud):
//     k_csv_len / k_pcd_len   the unit's text length (wave reduction)
//     k_csv_layout            unit byte offsets, file size
//   k_file_layout   offsets of every file of the batch in the packed output
//                   (and of every PNG's zlib staging area)
//   -- the host reads the totals and sizes the buffers --
//   k_png_emit      each row writes its bits at its offset: interior words
//                   with plain stores, the two words it may share with its
//                   neighbours with atomicOr (staging zeroed first)
//   k_png_ends      zlib + block header, end-of-block code, Adler-32
//   k_png_pack      one thread per 2-KiB IDAT chunk: copy into the file,
//                   chunk header, CRC-32 (LDS table); signature + IHDR and
//                   IEND at the ends
//   k_csv_emit / k_pcd_emit  each lane formats its text into the wave's LDS
//                   buffer; the wave stores the buffer coalesced
//
// Bandwidth (measured): the text kernels stream at 1.3-3.0 TB/s,
// the PNG passes at 0.4-0.9 TB/s; all of them together take a tenth of the
// time the packed files need to cross PCIe.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "csg_deflate.h"
#include "csg_encode.h"

namespace csg {

using namespace dfl;

namespace {

constexpr int kRowsPerBlock = 64;   // one wave of units per workgroup (one frame per workgroup)
// Work units: segments of rows, so that a batch offers tens of thousands of
// threads (one thread per 1080p row left the GPU mostly idle).
constexpr uint32_t kSegBytes = 512;  // PNG: raw row bytes per unit
constexpr uint32_t kSegVals = 64;    // CSV: values per unit

__host__ __device__ __forceinline__ uint32_t png_units(uint32_t W) { return (3u * W + kSegBytes - 1u) / kSegBytes; }
__host__ __device__ __forceinline__ uint32_t csv_units(uint32_t W) { return (W + kSegVals - 1u) / kSegVals; }

// The filtered PNG stream of unit k of an 8-bit RGB image row: raw bytes
// [k * kSegBytes, ...) each minus the byte one pixel (3 bytes) to its left (0
// before the row: filter type 1, Sub), preceded in unit 0 by the filter-type
// byte.  Units are tokenised independently: a run never crosses a unit
// boundary (a literal starts each unit; valid deflate, a few bytes larger).
// Rows with a 16-B aligned unit start stream 16-B loads, the next one issued
// before the current one is tokenised.
__device__ __forceinline__ uint32_t byte_of(const uint4& v, int t) {
  const uint32_t w = t < 4 ? v.x : t < 8 ? v.y : t < 12 ? v.z : v.w;
  return (w >> (8 * (t & 3))) & 255u;
}

template <class Sink>
__device__ __forceinline__ void png_unit_bytes(const uint8_t* row, uint32_t W, uint32_t k, Sink& sink) {
  const uint32_t j0 = k * kSegBytes, j1 = min(j0 + kSegBytes, 3u * W);
  if (k == 0) sink.push(1u);
  uint32_t j = j0;
  if (((reinterpret_cast<uintptr_t>(row) + j0) & 15u) == 0 && j + 16u <= j1) {
    uint4 prev = j0 ? *reinterpret_cast<const uint4*>(row + j0 - 16) : make_uint4(0u, 0u, 0u, 0u);
    uint4 cur = *reinterpret_cast<const uint4*>(row + j);
    for (; j + 16u <= j1; j += 16u) {
      const uint4 nxt = j + 32u <= j1 ? *reinterpret_cast<const uint4*>(row + j + 16) : cur;
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const uint32_t b = byte_of(cur, t), l = t >= 3 ? byte_of(cur, t - 3) : byte_of(prev, 13 + t);
        sink.push((b - l) & 255u);
      }
      prev = cur;
      cur = nxt;
    }
  }
  for (; j < j1; ++j) sink.push((uint32_t)(row[j] - (j >= 3u ? row[j - 3] : 0u)) & 255u);
}

// Adler sums of a byte stream starting from (0, 0), reduced lazily.
struct AdlerSums {
  uint64_t a = 0, b = 0;
  uint32_t pending = 0;
  __device__ __forceinline__ void add(uint32_t x) {
    a += x;
    b += a;
    if (++pending == 4096u) {
      a %= kAdlerMod;
      b %= kAdlerMod;
      pending = 0;
    }
  }
};

// ---------------------------------------------------------------------------
// PNG pass 1: histogram + Adler sums
// ---------------------------------------------------------------------------
// Unit u of a frame: row u / U, unit k = u % U of that row; its stream length.
__device__ __forceinline__ void png_unit(uint32_t u, uint32_t U, uint32_t& r, uint32_t& k) {
  r = u / U;
  k = u - r * U;
}
__device__ __forceinline__ uint32_t png_unit_len(uint32_t k, uint32_t W) {
  return min((k + 1u) * kSegBytes, 3u * W) - k * kSegBytes + (k == 0 ? 1u : 0u);
}

__global__ __launch_bounds__(kRowsPerBlock) void k_png_scan(const uint8_t* __restrict__ img, uint32_t W, uint32_t H,
                                                            EncPng* __restrict__ png, uint2* __restrict__ usum) {
  __shared__ uint32_t hist[kLitCodes];
  const uint32_t f = blockIdx.y, U = png_units(W), u = blockIdx.x * kRowsPerBlock + threadIdx.x;
  for (uint32_t s = threadIdx.x; s < (uint32_t)kLitCodes; s += kRowsPerBlock) hist[s] = 0;
  __syncthreads();
  if (u < H * U) {
    uint32_t r, k;
    png_unit(u, U, r, k);
    AdlerSums ad;
    auto lit = [&](uint32_t b) { atomicAdd(&hist[b], 1u); };
    auto match = [&](uint32_t len) {
      uint32_t sym, ne, ex;
      length_code(len, sym, ne, ex);
      atomicAdd(&hist[sym], 1u);
    };
    struct Sink {
      RunTokenizer<decltype(lit)&, decltype(match)&> tok;
      AdlerSums* ad;
      __device__ void push(uint32_t x) {
        ad->add(x);
        tok.push(x);
      }
    } sink{{lit, match}, &ad};
    png_unit_bytes(img + ((size_t)f * H + r) * (size_t)W * 3u, W, k, sink);
    sink.tok.finish();
    usum[(size_t)f * H * U + u] = make_uint2((uint32_t)(ad.a % kAdlerMod), (uint32_t)(ad.b % kAdlerMod));
  }
  __syncthreads();
  for (uint32_t s = threadIdx.x; s < (uint32_t)kLitCodes; s += kRowsPerBlock)
    if (hist[s]) atomicAdd(&png[f].hist[s], hist[s]);
}

// ---------------------------------------------------------------------------
// PNG pass 2: codes and header (one workgroup of 256 threads per frame)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_png_codes(EncPng* __restrict__ png, const uint2* __restrict__ rowsum,
                                                   uint32_t W, uint32_t H) {
  __shared__ uint32_t freq[kLitCodes];
  __shared__ uint16_t sorted[kLitCodes];
  __shared__ uint32_t work[kLitCodes];
  __shared__ uint8_t len[kLitCodes + 1];      // + the one distance code
  __shared__ uint32_t code[kLitCodes];
  __shared__ uint16_t tok[kLitCodes + 1];
  __shared__ uint32_t m_used;
  const uint32_t f = blockIdx.x, t = threadIdx.x;
  EncPng& P = png[f];
  for (uint32_t s = t; s < (uint32_t)kLitCodes; s += 256) {
    freq[s] = s == kEob ? 1u : P.hist[s];
    len[s] = 0;
  }
  if (t == 0) m_used = 0;
  __syncthreads();
  // rank of each used symbol in ascending (frequency, symbol) order
  for (uint32_t s = t; s < (uint32_t)kLitCodes; s += 256) {
    const uint32_t fs = freq[s];
    if (!fs) continue;
    uint32_t rank = 0;
    for (uint32_t q = 0; q < (uint32_t)kLitCodes; ++q) {
      const uint32_t fq = freq[q];
      rank += (fq && (fq < fs || (fq == fs && q < s))) ? 1u : 0u;
    }
    sorted[rank] = (uint16_t)s;
    atomicAdd(&m_used, 1u);
  }
  __syncthreads();
  if (t == 0) {
    const int m = (int)m_used;   // >= 2: the filter byte of row 0 and the end-of-block code
    huff_lengths(freq, sorted, m, kMaxBits, len, work);
    canonical_codes(len, kLitCodes, code);
    int hlit = kLitCodes;
    while (hlit > 257 && len[hlit - 1] == 0) --hlit;
    len[hlit] = 1;               // one distance code (distance 1), length 1
    const int ntok = cl_tokens(len, hlit + 1, tok);
    uint32_t clf[kClCodes] = {0};
    for (int k = 0; k < ntok; ++k) ++clf[tok[k] & 31u];
    uint16_t cls[kClCodes];
    int cm = 0;
    for (uint32_t s = 0; s < (uint32_t)kClCodes; ++s) {
      if (!clf[s]) continue;
      int k = cm++;   // insertion into ascending (frequency, symbol) order
      while (k > 0 && clf[cls[k - 1]] > clf[s]) {
        cls[k] = cls[k - 1];
        --k;
      }
      cls[k] = (uint16_t)s;
    }
    uint8_t cll[kClCodes] = {0};
    uint32_t clw[kClCodes];
    huff_lengths(clf, cls, cm, kMaxClBits, cll, clw);
    if (cm == 1) cll[cls[0] == 0 ? 1 : 0] = 1;   // the code-length code must be complete
    uint32_t clc[kClCodes];
    canonical_codes(cll, kClCodes, clc);
    int hclen = kClCodes;
    while (hclen > 4 && cll[cl_order(hclen - 1)] == 0) --hclen;
    for (uint32_t k = 0; k < kMaxHeaderWords; ++k) P.hdr[k] = 0;
    BitBuf bb{P.hdr, 0};
    bb.put(0x78u, 8);            // zlib: deflate, 32 KiB window
    bb.put(0x01u, 8);            // FCHECK (0x7801 % 31 == 0), no dictionary
    bb.put(1u, 1);               // BFINAL
    bb.put(2u, 2);               // BTYPE = dynamic Huffman
    bb.put((uint32_t)(hlit - 257), 5);
    bb.put(0u, 5);               // HDIST - 1
    bb.put((uint32_t)(hclen - 4), 4);
    for (int k = 0; k < hclen; ++k) bb.put(cll[cl_order(k)], 3);
    for (int k = 0; k < ntok; ++k) {
      const uint32_t sym = tok[k] & 31u, ex = (uint32_t)tok[k] >> 8;
      bb.put(clc[sym] & 0xFFFFu, clc[sym] >> 16);
      bb.put(ex, cl_extra_bits(sym));
    }
    P.hdr_bits = bb.nbits;
    for (uint32_t s = 0; s < (uint32_t)kLitCodes; ++s) P.code[s] = code[s];
  }
  // Adler-32 of the whole filtered stream: each thread folds a contiguous run
  // of units in order, then an ordered tree over the threads (the fold of
  // (a, b, length) is associative)
  __shared__ uint32_t sa[256], sb[256];
  __shared__ uint64_t sl[256];
  const uint32_t U = png_units(W), n = H * U, per = (n + 255u) / 256u, lo = t * per, hi = min(n, lo + per);
  uint32_t a = 0, b = 0;
  uint64_t l = 0;
  for (uint32_t u = lo; u < hi; ++u) {
    const uint2 v = rowsum[(size_t)f * n + u];
    const uint32_t len = png_unit_len(u % U, W);
    adler_cat(a, b, v.x, v.y, len);
    l += len;
  }
  sa[t] = a;
  sb[t] = b;
  sl[t] = l;
  __syncthreads();
  for (uint32_t o = 1; o < 256u; o <<= 1) {
    if ((t & (2u * o - 1u)) == 0 && t + o < 256u) {
      uint32_t a1 = sa[t], b1 = sb[t];
      adler_cat(a1, b1, sa[t + o], sb[t + o], sl[t + o]);
      sa[t] = a1;
      sb[t] = b1;
      sl[t] += sl[t + o];
    }
    __syncthreads();
  }
  if (t == 0) {
    uint32_t A = 1, B = 0;   // the stream's Adler-32 starts from (1, 0)
    adler_cat(A, B, sa[0], sb[0], sl[0]);
    P.adler = (B << 16) | A;
  }
}

// ---------------------------------------------------------------------------
// PNG pass 3: bits per row
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kRowsPerBlock) void k_png_bits(const uint8_t* __restrict__ img, uint32_t W, uint32_t H,
                                                            const EncPng* __restrict__ png, uint32_t* __restrict__ ubits) {
  __shared__ uint8_t clen[kLitCodes];
  const uint32_t f = blockIdx.y, U = png_units(W), u = blockIdx.x * kRowsPerBlock + threadIdx.x;
  for (uint32_t s = threadIdx.x; s < (uint32_t)kLitCodes; s += kRowsPerBlock) clen[s] = (uint8_t)(png[f].code[s] >> 16);
  __syncthreads();
  if (u >= H * U) return;
  uint32_t r, k;
  png_unit(u, U, r, k);
  uint32_t bits = 0;
  auto lit = [&](uint32_t b) { bits += clen[b]; };
  auto match = [&](uint32_t len) {
    uint32_t sym, ne, ex;
    length_code(len, sym, ne, ex);
    bits += clen[sym] + ne + 1u;   // + the 1-bit distance code
  };
  struct Sink {
    RunTokenizer<decltype(lit)&, decltype(match)&> tok;
    __device__ void push(uint32_t x) { tok.push(x); }
  } sink{{lit, match}};
  png_unit_bytes(img + ((size_t)f * H + r) * (size_t)W * 3u, W, k, sink);
  sink.tok.finish();
  ubits[(size_t)f * H * U + u] = bits;
}

// exclusive scan of n values (in place) over a 256-thread block; returns the total
__device__ uint32_t block_scan_inplace(uint32_t* v, uint32_t n, uint32_t* sh) {
  const uint32_t t = threadIdx.x, per = (n + 255u) / 256u, lo = t * per, hi = min(n, lo + per);
  uint32_t s = 0;
  for (uint32_t i = lo; i < hi; ++i) s += v[i];
  sh[t] = s;
  __syncthreads();
  for (uint32_t o = 1; o < 256u; o <<= 1) {
    const uint32_t x = t >= o ? sh[t - o] : 0u;
    __syncthreads();
    sh[t] += x;
    __syncthreads();
  }
  uint32_t run = sh[t] - s;
  const uint32_t total = sh[255];
  for (uint32_t i = lo; i < hi; ++i) {
    const uint32_t x = v[i];
    v[i] = run;
    run += x;
  }
  __syncthreads();
  return total;
}

// ---------------------------------------------------------------------------
// PNG pass 4: row offsets, sizes
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_png_layout(EncPng* __restrict__ png, uint32_t* __restrict__ ubits, uint32_t n,
                                                    uint64_t* __restrict__ fsize, uint32_t nk, uint32_t kslot) {
  __shared__ uint32_t sh[256];
  const uint32_t f = blockIdx.x;
  EncPng& P = png[f];
  const uint32_t total = block_scan_inplace(ubits + (size_t)f * n, n, sh);
  if (threadIdx.x == 0) {
    const uint32_t eob_len = P.code[kEob] >> 16;
    P.eob_pos = P.hdr_bits + total;
    const uint32_t zbits = P.eob_pos + eob_len;
    P.zbytes = (zbits + 7u) / 8u + 4u;
    const uint32_t nch = (P.zbytes + kIdatBytes - 1u) / kIdatBytes;
    fsize[(size_t)f * nk + kslot] = 8ull + 25ull + 12ull * nch + P.zbytes + 12ull;
  }
}

// ---------------------------------------------------------------------------
// Text files (depth CSV, point-cloud TXT): one wave per unit of 64 items
// ---------------------------------------------------------------------------
// A unit is 64 consecutive pixels of one row (the row's last unit may be
// short); lane i owns pixel i.  The length pass reduces the lanes' text
// lengths to the unit's; the emit pass scans them, each lane formats its text
// into the wave's LDS buffer at its offset, and the wave copies the buffer to
// the file with coalesced dword stores (the unaligned ends as bytes).  The
// buffer holds the texts of the longest possible length: 64 CSV values, or
// the point lines of half a wave (k_pcd_emit runs the two halves in turn).
constexpr uint32_t kTxtWaves = 4;          // units per 256-thread workgroup
constexpr uint32_t kCsvBuf = 64u * (kMaxF6Chars + 1);              // 3.1 KB per wave: a value and its separator
constexpr uint32_t kPcdBuf = 32u * kMaxPcdLine + kPcdHeaderBytes;   // 5.8 KB per wave

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t lane, uint32_t& total) {
  uint32_t s = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(s, o, 64);
    if (lane >= (uint32_t)o) s += t;
  }
  total = __shfl(s, 63, 64);
  return s - v;
}

// Copy n bytes of the wave's LDS text to out + pos: head and tail bytes with
// byte stores (those dwords are shared with the neighbouring units), the
// dwords between with one coalesced store per lane and round.
__device__ __forceinline__ void wave_copy_out(const uint32_t* buf, uint32_t n, uint8_t* out, uint64_t pos,
                                              uint32_t lane) {
  const uint8_t* bb = reinterpret_cast<const uint8_t*>(buf);
  const uint64_t end = pos + n, a0 = min((pos + 3u) & ~3ull, end), a1 = max(end & ~3ull, a0);
  const uint32_t head = (uint32_t)(a0 - pos), tail = (uint32_t)(end - a1);
  if (lane < head) out[pos + lane] = bb[lane];
  if (lane < tail) out[a1 + lane] = bb[(uint32_t)(a1 - pos) + lane];
  const uint32_t nw = (uint32_t)((a1 - a0) >> 2);
  uint32_t* ow = reinterpret_cast<uint32_t*>(out + a0);
  for (uint32_t j = lane; j < nw; j += 64u) {
    const uint32_t o = head + 4u * j, w = o >> 2, sh = o & 3u;
    const uint32_t lo = buf[w], hi = buf[w + 1];
    ow[j] = sh ? __builtin_amdgcn_alignbyte(hi, lo, sh) : lo;
  }
}

// Unit u of a frame: row u / V, pixels [(u % V) * 64, ...) of it.
__device__ __forceinline__ void txt_unit(uint32_t u, uint32_t V, uint32_t W, uint32_t& r, uint32_t& x0, uint32_t& x1) {
  r = u / V;
  x0 = (u - r * V) * kSegVals;
  x1 = min(x0 + kSegVals, W);
}

// Depth CSV: each value followed by a space, the row's last by a newline.
__global__ __launch_bounds__(64 * kTxtWaves) void k_csv_len(const float* __restrict__ depth, uint32_t W, uint32_t H,
                                                            uint32_t* __restrict__ ulen) {
  const uint32_t f = blockIdx.y, V = csv_units(W), lane = threadIdx.x & 63u;
  const uint32_t u = blockIdx.x * kTxtWaves + (threadIdx.x >> 6);
  if (u >= H * V) return;
  uint32_t r, x0, x1;
  txt_unit(u, V, W, r, x0, x1);
  const uint32_t x = x0 + lane;
  const uint32_t n = x < x1 ? (uint32_t)fmt6f_len(depth[((size_t)f * H + r) * W + x]) + 1u : 0u;
  const uint32_t tot = wave_sum(n);
  if (lane == 0) ulen[(size_t)f * H * V + u] = tot;
}

// Point-cloud TXT: one line per pixel with a point, in row-major order; the
// frame's unit 0 also carries the 12-byte header line.
__global__ __launch_bounds__(64 * kTxtWaves) void k_pcd_len(const float* __restrict__ pts, const uint8_t* __restrict__ rgb,
                                                            uint32_t W, uint32_t H, uint32_t* __restrict__ ulen) {
  const uint32_t f = blockIdx.y, V = csv_units(W), lane = threadIdx.x & 63u;
  const uint32_t u = blockIdx.x * kTxtWaves + (threadIdx.x >> 6);
  if (u >= H * V) return;
  uint32_t r, x0, x1;
  txt_unit(u, V, W, r, x0, x1);
  const uint32_t x = x0 + lane;
  uint32_t n = 0;
  if (x < x1) {
    const size_t px = ((size_t)f * H + r) * W + x;
    const float X = pts[3 * px], Y = pts[3 * px + 1], Z = pts[3 * px + 2];
    if (pcd_valid(X, Y, Z)) n = (uint32_t)pcd_line_len(X, Y, Z, rgb[3 * px], rgb[3 * px + 1], rgb[3 * px + 2]);
  }
  const uint32_t tot = wave_sum(n);
  if (lane == 0) ulen[(size_t)f * H * V + u] = tot + (u == 0 ? kPcdHeaderBytes : 0u);
}

__global__ __launch_bounds__(256) void k_csv_layout(uint32_t* __restrict__ ulen, uint32_t n, uint64_t* __restrict__ fsize,
                                                    uint32_t nk, uint32_t kslot) {
  __shared__ uint32_t sh[256];
  const uint32_t f = blockIdx.x;
  const uint32_t total = block_scan_inplace(ulen + (size_t)f * n, n, sh);
  if (threadIdx.x == 0) fsize[(size_t)f * nk + kslot] = total;
}

// Offsets of the batch's files in the packed output (foff[n_files + 1]) and
// of each PNG frame's zlib staging area (zoff: kind a frames, then kind b
// frames, then the total; 256-B aligned).  A few hundred entries: one thread.
__global__ void k_file_layout(const uint64_t* __restrict__ fsize, uint32_t n_files, uint64_t* __restrict__ foff,
                              const EncPng* __restrict__ png_a, const EncPng* __restrict__ png_b, uint32_t F,
                              uint64_t* __restrict__ zoff) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint64_t run = 0;
  for (uint32_t k = 0; k < n_files; ++k) {
    foff[k] = run;
    run += fsize[k];
  }
  foff[n_files] = run;
  uint64_t z = 0;
  for (uint32_t k = 0; k < 2u * F; ++k) {
    zoff[k] = z;
    const EncPng* p = k < F ? png_a : png_b;
    if (p) z += ((uint64_t)p[k < F ? k : k - F].zbytes + 255u) & ~255ull;
  }
  zoff[2u * F] = z;
}

// ---------------------------------------------------------------------------
// PNG emission
// ---------------------------------------------------------------------------
// LSB-first bits into zeroed staging words from bit `pos`: the first word
// (possibly shared with the previous row) and the last (possibly shared with
// the next) with atomicOr, words in between with plain stores.
struct WordBits {
  uint32_t* w;
  uint64_t acc;
  uint32_t n, wi;
  bool first;
  __device__ void init(uint32_t* words, uint32_t pos) {
    w = words;
    wi = pos >> 5;
    n = pos & 31u;
    acc = 0;
    first = true;
  }
  __device__ __forceinline__ void put(uint32_t v, uint32_t len) {
    acc |= (uint64_t)v << n;
    n += len;
    if (n >= 32u) {
      const uint32_t word = (uint32_t)acc;
      if (first) atomicOr(&w[wi], word);
      else w[wi] = word;
      first = false;
      ++wi;
      acc >>= 32;
      n -= 32u;
    }
  }
  __device__ void finish() {
    if (n) atomicOr(&w[wi], (uint32_t)acc);
  }
};

__global__ __launch_bounds__(kRowsPerBlock) void k_png_emit(const uint8_t* __restrict__ img, uint32_t W, uint32_t H,
                                                            const EncPng* __restrict__ png,
                                                            const uint32_t* __restrict__ uoff, uint8_t* zbuf,
                                                            const uint64_t* __restrict__ zbase) {
  __shared__ uint32_t code[kLitCodes];
  const uint32_t f = blockIdx.y, U = png_units(W), u = blockIdx.x * kRowsPerBlock + threadIdx.x;
  for (uint32_t s = threadIdx.x; s < (uint32_t)kLitCodes; s += kRowsPerBlock) code[s] = png[f].code[s];
  __syncthreads();
  if (u >= H * U) return;
  uint32_t r, k;
  png_unit(u, U, r, k);
  uint32_t* words = reinterpret_cast<uint32_t*>(zbuf + zbase[f]);
  WordBits wb;
  wb.init(words, png[f].hdr_bits + uoff[(size_t)f * H * U + u]);
  auto lit = [&](uint32_t b) { wb.put(code[b] & 0xFFFFu, code[b] >> 16); };
  auto match = [&](uint32_t len) {
    uint32_t sym, ne, ex;
    length_code(len, sym, ne, ex);
    wb.put(code[sym] & 0xFFFFu, code[sym] >> 16);
    wb.put(ex, ne);
    wb.put(0u, 1u);   // distance code 0 (distance 1), code "0"
  };
  struct Sink {
    RunTokenizer<decltype(lit)&, decltype(match)&> tok;
    __device__ void push(uint32_t x) { tok.push(x); }
  } sink{{lit, match}};
  png_unit_bytes(img + ((size_t)f * H + r) * (size_t)W * 3u, W, k, sink);
  sink.tok.finish();
  wb.finish();
}

// header words, end-of-block code, Adler-32 (big-endian) after the padding
__global__ __launch_bounds__(64) void k_png_ends(const EncPng* __restrict__ png, uint8_t* zbuf,
                                                 const uint64_t* __restrict__ zbase) {
  const uint32_t f = blockIdx.x;
  const EncPng& P = png[f];
  uint32_t* words = reinterpret_cast<uint32_t*>(zbuf + zbase[f]);
  const uint32_t nh = (P.hdr_bits + 31u) / 32u;
  for (uint32_t k = threadIdx.x; k < nh; k += 64) atomicOr(&words[k], P.hdr[k]);
  if (threadIdx.x == 0) {
    const uint32_t c = P.code[kEob], l = c >> 16, pos = P.eob_pos;
    const uint64_t v = (uint64_t)(c & 0xFFFFu) << (pos & 31u);
    atomicOr(&words[pos >> 5], (uint32_t)v);
    if ((pos & 31u) + l > 32u) atomicOr(&words[(pos >> 5) + 1], (uint32_t)(v >> 32));
    const uint32_t at = P.zbytes - 4u;   // byte index of the Adler-32
    const uint32_t be = __builtin_bswap32(P.adler);
    const uint64_t sv = (uint64_t)be << (8u * (at & 3u));
    atomicOr(&words[at >> 2], (uint32_t)sv);
    if (at & 3u) atomicOr(&words[(at >> 2) + 1], (uint32_t)(sv >> 32));
  }
}

// Bytes to an arbitrary offset: byte stores up to a dword boundary, then
// whole dwords, the tail again as bytes.
struct ByteOut {
  uint8_t* base;
  uint64_t pos;
  uint32_t acc, na;
  __device__ void init(uint8_t* b, uint64_t p) {
    base = b;
    pos = p;
    acc = 0;
    na = 0;
  }
  __device__ __forceinline__ void put(uint32_t c) {
    if (na == 0 && (pos & 3u)) {
      base[pos++] = (uint8_t)c;
      return;
    }
    acc |= (c & 255u) << (8u * na);
    ++pos;
    if (++na == 4u) {
      *reinterpret_cast<uint32_t*>(base + pos - 4u) = acc;
      acc = 0;
      na = 0;
    }
  }
  __device__ void be32(uint32_t v) {
    put(v >> 24);
    put((v >> 16) & 255u);
    put((v >> 8) & 255u);
    put(v & 255u);
  }
  __device__ void finish() {
    for (uint32_t k = 0; k < na; ++k) base[pos - na + k] = (uint8_t)(acc >> (8u * k));
    na = 0;
    acc = 0;
  }
};

struct Crc {
  const uint32_t* T;
  uint32_t c;
  __device__ __forceinline__ void add(uint32_t b) { c = T[(c ^ b) & 255u] ^ (c >> 8); }
};

__global__ __launch_bounds__(64) void k_png_pack(const EncPng* __restrict__ png, const uint8_t* __restrict__ zbuf,
                                                 const uint64_t* __restrict__ zbase, uint8_t* out,
                                                 const uint64_t* __restrict__ foff, uint32_t W, uint32_t H, uint32_t nk,
                                                 uint32_t kslot) {
  __shared__ uint32_t T[256];
  for (uint32_t k = threadIdx.x; k < 256u; k += 64) T[k] = crc_entry(k);
  __syncthreads();
  const uint32_t f = blockIdx.y, ch = blockIdx.x * 64u + threadIdx.x;
  const EncPng& P = png[f];
  const uint32_t zb = P.zbytes, nch = (zb + kIdatBytes - 1u) / kIdatBytes;
  if (ch >= nch) return;
  uint8_t* file = out + foff[(size_t)f * nk + kslot];
  const uint32_t n = min(kIdatBytes, zb - ch * kIdatBytes);
  ByteOut o;
  if (ch == 0) {   // signature + IHDR
    o.init(file, 0);
    const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    for (int k = 0; k < 8; ++k) o.put(sig[k]);
    o.be32(13u);
    Crc c{T, 0xFFFFFFFFu};
    const uint8_t ihdr[17] = {'I', 'H', 'D', 'R', (uint8_t)(W >> 24), (uint8_t)(W >> 16), (uint8_t)(W >> 8), (uint8_t)W,
                              (uint8_t)(H >> 24), (uint8_t)(H >> 16), (uint8_t)(H >> 8), (uint8_t)H, 8, 2, 0, 0, 0};
    for (int k = 0; k < 17; ++k) {
      o.put(ihdr[k]);
      c.add(ihdr[k]);
    }
    o.be32(c.c ^ 0xFFFFFFFFu);
    o.finish();
  }
  const uint64_t at = 33ull + (uint64_t)ch * (kIdatBytes + 12u);
  o.init(file, at);
  o.be32(n);
  Crc c{T, 0xFFFFFFFFu};
  const uint8_t idat[4] = {'I', 'D', 'A', 'T'};
  for (int k = 0; k < 4; ++k) {
    o.put(idat[k]);
    c.add(idat[k]);
  }
  const uint32_t* src = reinterpret_cast<const uint32_t*>(zbuf + zbase[f] + (size_t)ch * kIdatBytes);
  const uint32_t nw = n >> 2;
  for (uint32_t k = 0; k < nw; ++k) {
    const uint32_t v = src[k];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const uint32_t b = (v >> (8 * s)) & 255u;
      o.put(b);
      c.add(b);
    }
  }
  if (n & 3u) {
    const uint32_t v = src[nw];
    for (uint32_t s = 0; s < (n & 3u); ++s) {
      const uint32_t b = (v >> (8u * s)) & 255u;
      o.put(b);
      c.add(b);
    }
  }
  o.be32(c.c ^ 0xFFFFFFFFu);
  if (ch == nch - 1u) {   // IEND
    o.be32(0u);
    const uint8_t iend[8] = {'I', 'E', 'N', 'D', 0xAE, 0x42, 0x60, 0x82};
    for (int k = 0; k < 8; ++k) o.put(iend[k]);
  }
  o.finish();
}

__global__ __launch_bounds__(64 * kTxtWaves) void k_csv_emit(const float* __restrict__ depth, uint32_t W, uint32_t H,
                                                             const uint32_t* __restrict__ uoff, uint8_t* out,
                                                             const uint64_t* __restrict__ foff, uint32_t nk,
                                                             uint32_t kslot) {
  __shared__ uint32_t tbuf[kTxtWaves][kCsvBuf / 4 + 1];
  const uint32_t f = blockIdx.y, V = csv_units(W), lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t u = blockIdx.x * kTxtWaves + wv;
  if (u >= H * V) return;
  uint32_t r, x0, x1;
  txt_unit(u, V, W, r, x0, x1);
  const uint32_t x = x0 + lane;
  const float d = x < x1 ? depth[((size_t)f * H + r) * W + x] : 0.0f;
  const uint32_t n = x < x1 ? (uint32_t)fmt6f_len(d) + 1u : 0u;
  uint32_t total;
  const uint32_t off = wave_excl_scan(n, lane, total);
  const uint64_t pos = foff[(size_t)f * nk + kslot] + uoff[(size_t)f * H * V + u];
  const char sep = x + 1u < W ? ' ' : '\n';
  char* t = reinterpret_cast<char*>(tbuf[wv]);
  if (n) {
    fmt6f(d, t + off);
    t[off + n - 1u] = sep;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  wave_copy_out(tbuf[wv], total, out, pos, lane);
}

__global__ __launch_bounds__(64 * kTxtWaves) void k_pcd_emit(const float* __restrict__ pts, const uint8_t* __restrict__ rgb,
                                                             uint32_t W, uint32_t H, const uint32_t* __restrict__ uoff,
                                                             uint8_t* out, const uint64_t* __restrict__ foff,
                                                             uint32_t nk, uint32_t kslot) {
  __shared__ uint32_t tbuf[kTxtWaves][kPcdBuf / 4 + 1];
  const uint32_t f = blockIdx.y, V = csv_units(W), lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t u = blockIdx.x * kTxtWaves + wv;
  if (u >= H * V) return;
  uint32_t r, x0, x1;
  txt_unit(u, V, W, r, x0, x1);
  const uint32_t x = x0 + lane;
  float X = 0.0f, Y = 0.0f, Z = 0.0f;
  uint32_t R = 0, G = 0, B = 0, n = 0;
  if (x < x1) {
    const size_t px = ((size_t)f * H + r) * W + x;
    X = pts[3 * px];
    Y = pts[3 * px + 1];
    Z = pts[3 * px + 2];
    R = rgb[3 * px];
    G = rgb[3 * px + 1];
    B = rgb[3 * px + 2];
    if (pcd_valid(X, Y, Z)) n = (uint32_t)pcd_line_len(X, Y, Z, R, G, B);
  }
  const uint32_t hdr = u == 0 ? kPcdHeaderBytes : 0u;
  uint32_t total;
  const uint32_t off = wave_excl_scan(n, lane, total) + hdr;
  total += hdr;
  const uint64_t pos = foff[(size_t)f * nk + kslot] + uoff[(size_t)f * H * V + u];
  // lanes 0-31 (and the header), then lanes 32-63: each half's text is a
  // contiguous range of the unit's
  const uint32_t split = __shfl(off, 32, 64);
  char* t = reinterpret_cast<char*>(tbuf[wv]);
#pragma unroll
  for (uint32_t h = 0; h < 2; ++h) {
    const uint32_t lo = h ? split : 0u, hi = h ? total : split;
    if ((lane >> 5) == h) {
      if (lane < hdr) t[lane] = pcd_header_byte(lane);
      if (n) pcd_line(X, Y, Z, R, G, B, t + (off - lo));
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    wave_copy_out(tbuf[wv], hi - lo, out, pos + lo, lane);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// ---------------------------------------------------------------------------
// depth statistics of the quality log (csg_outputs.depth_stats)
// ---------------------------------------------------------------------------
constexpr uint32_t kStatBlocks = 64;
struct DepthPartial {
  double sum;
  uint32_t valid, zero, inf, mn, mx, pad;
};

__global__ __launch_bounds__(256) void k_depth_stats(const float* __restrict__ depth, uint32_t npx,
                                                     DepthPartial* __restrict__ part) {
  const uint32_t f = blockIdx.y;
  const float* d = depth + (size_t)f * npx;
  double sum = 0.0;
  uint32_t valid = 0, zero = 0, inf = 0, mn = 0xFFFFFFFFu, mx = 0u;
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < npx; i += kStatBlocks * 256u) {
    const float v = d[i];
    const uint32_t u = __float_as_uint(v);
    if (v > 0.0f && v < INFINITY) {
      ++valid;
      sum += (double)v;
      mn = min(mn, u);
      mx = max(mx, u);
    }
    zero += v == 0.0f ? 1u : 0u;
    inf += (u & 0x7FFFFFFFu) == 0x7F800000u ? 1u : 0u;
  }
  __shared__ DepthPartial sh[256];
  sh[threadIdx.x] = DepthPartial{sum, valid, zero, inf, mn, mx, 0};
  __syncthreads();
  for (uint32_t o = 128; o > 0; o >>= 1) {   // fixed tree order: deterministic
    if (threadIdx.x < o) {
      DepthPartial& a = sh[threadIdx.x];
      const DepthPartial& b = sh[threadIdx.x + o];
      a.sum += b.sum;
      a.valid += b.valid;
      a.zero += b.zero;
      a.inf += b.inf;
      a.mn = min(a.mn, b.mn);
      a.mx = max(a.mx, b.mx);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) part[(size_t)f * kStatBlocks + blockIdx.x] = sh[0];
}

__global__ void k_depth_stats_final(const DepthPartial* __restrict__ part, uint32_t F, double* __restrict__ out) {
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= F) return;
  DepthPartial a{0.0, 0, 0, 0, 0xFFFFFFFFu, 0u, 0};
  for (uint32_t b = 0; b < kStatBlocks; ++b) {
    const DepthPartial& p = part[(size_t)f * kStatBlocks + b];
    a.sum += p.sum;
    a.valid += p.valid;
    a.zero += p.zero;
    a.inf += p.inf;
    a.mn = min(a.mn, p.mn);
    a.mx = max(a.mx, p.mx);
  }
  double* o = out + (size_t)f * 6;
  o[0] = a.valid;
  o[1] = a.zero;
  o[2] = a.inf;
  o[3] = a.sum;
  o[4] = a.valid ? (double)__uint_as_float(a.mn) : 0.0;
  o[5] = a.valid ? (double)__uint_as_float(a.mx) : 0.0;
}

}  // namespace

// ---------------------------------------------------------------------------
// launchers (csg_encode.h)
// ---------------------------------------------------------------------------
uint32_t png_units_per_frame(uint32_t W, uint32_t H) { return png_units(W) * H; }
uint32_t csv_units_per_frame(uint32_t W, uint32_t H) { return csv_units(W) * H; }

void launch_png_sizes(const uint8_t* img, uint32_t W, uint32_t H, uint32_t F, EncPng* png, uint2* usum,
                      uint32_t* ubits, uint64_t* fsize, uint32_t nk, uint32_t kslot, hipStream_t st) {
  const uint32_t n = png_units_per_frame(W, H);
  const dim3 units((n + kRowsPerBlock - 1) / kRowsPerBlock, F);
  (void)hipMemsetAsync(png, 0, sizeof(EncPng) * F, st);
  hipLaunchKernelGGL(k_png_scan, units, dim3(kRowsPerBlock), 0, st, img, W, H, png, usum);
  hipLaunchKernelGGL(k_png_codes, dim3(F), dim3(256), 0, st, png, usum, W, H);
  hipLaunchKernelGGL(k_png_bits, units, dim3(kRowsPerBlock), 0, st, img, W, H, png, ubits);
  hipLaunchKernelGGL(k_png_layout, dim3(F), dim3(256), 0, st, png, ubits, n, fsize, nk, kslot);
}

void launch_csv_sizes(const float* depth, uint32_t W, uint32_t H, uint32_t F, uint32_t* ulen, uint64_t* fsize,
                      uint32_t nk, uint32_t kslot, hipStream_t st) {
  const uint32_t n = csv_units_per_frame(W, H);
  const dim3 units((n + kTxtWaves - 1) / kTxtWaves, F);
  hipLaunchKernelGGL(k_csv_len, units, dim3(64 * kTxtWaves), 0, st, depth, W, H, ulen);
  hipLaunchKernelGGL(k_csv_layout, dim3(F), dim3(256), 0, st, ulen, n, fsize, nk, kslot);
}

void launch_pcd_sizes(const float* points, const uint8_t* rgb, uint32_t W, uint32_t H, uint32_t F, uint32_t* ulen,
                      uint64_t* fsize, uint32_t nk, uint32_t kslot, hipStream_t st) {
  const uint32_t n = csv_units_per_frame(W, H);
  const dim3 units((n + kTxtWaves - 1) / kTxtWaves, F);
  hipLaunchKernelGGL(k_pcd_len, units, dim3(64 * kTxtWaves), 0, st, points, rgb, W, H, ulen);
  hipLaunchKernelGGL(k_csv_layout, dim3(F), dim3(256), 0, st, ulen, n, fsize, nk, kslot);
}

void launch_file_layout(const uint64_t* fsize, uint32_t n_files, uint64_t* foff, const EncPng* png_a,
                        const EncPng* png_b, uint32_t F, uint64_t* zoff, hipStream_t st) {
  hipLaunchKernelGGL(k_file_layout, dim3(1), dim3(64), 0, st, fsize, n_files, foff, png_a, png_b, F, zoff);
}

void launch_png_emit(const uint8_t* img, uint32_t W, uint32_t H, uint32_t F, const EncPng* png, const uint32_t* rowoff,
                     uint8_t* zbuf, const uint64_t* zbase, uint8_t* out, const uint64_t* foff, uint32_t nk,
                     uint32_t kslot, hipStream_t st) {
  const uint32_t n = png_units_per_frame(W, H);
  hipLaunchKernelGGL(k_png_emit, dim3((n + kRowsPerBlock - 1) / kRowsPerBlock, F), dim3(kRowsPerBlock), 0, st, img, W,
                     H, png, rowoff, zbuf, zbase);
  hipLaunchKernelGGL(k_png_ends, dim3(F), dim3(64), 0, st, png, zbuf, zbase);
  // chunks per frame: at most the worst-case stream size / kIdatBytes
  const uint64_t max_z = (uint64_t)H * (3ull * W + 1ull) * 2ull + 65536ull;
  const uint32_t max_ch = (uint32_t)((max_z + kIdatBytes - 1) / kIdatBytes);
  hipLaunchKernelGGL(k_png_pack, dim3((max_ch + 63) / 64, F), dim3(64), 0, st, png, zbuf, zbase, out, foff, W, H, nk,
                     kslot);
}

size_t depth_stats_scratch_bytes(uint32_t F) { return sizeof(DepthPartial) * kStatBlocks * F; }

void launch_depth_stats(const float* depth, uint32_t npx, uint32_t F, void* scratch, double* out, hipStream_t st) {
  DepthPartial* part = static_cast<DepthPartial*>(scratch);
  hipLaunchKernelGGL(k_depth_stats, dim3(kStatBlocks, F), dim3(256), 0, st, depth, npx, part);
  hipLaunchKernelGGL(k_depth_stats_final, dim3((F + 63) / 64), dim3(64), 0, st, part, F, out);
}

void launch_csv_emit(const float* depth, uint32_t W, uint32_t H, uint32_t F, const uint32_t* rowoff, uint8_t* out,
                     const uint64_t* foff, uint32_t nk, uint32_t kslot, hipStream_t st) {
  const uint32_t n = csv_units_per_frame(W, H);
  hipLaunchKernelGGL(k_csv_emit, dim3((n + kTxtWaves - 1) / kTxtWaves, F), dim3(64 * kTxtWaves), 0, st, depth, W, H,
                     rowoff, out, foff, nk, kslot);
}

void launch_pcd_emit(const float* points, const uint8_t* rgb, uint32_t W, uint32_t H, uint32_t F, const uint32_t* rowoff,
                     uint8_t* out, const uint64_t* foff, uint32_t nk, uint32_t kslot, hipStream_t st) {
  const uint32_t n = csv_units_per_frame(W, H);
  hipLaunchKernelGGL(k_pcd_emit, dim3((n + kTxtWaves - 1) / kTxtWaves, F), dim3(64 * kTxtWaves), 0, st, points, rgb,
                     W, H, rowoff, out, foff, nk, kslot);
}

}  // namespace csg
