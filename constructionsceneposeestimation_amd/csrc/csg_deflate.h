// csg_deflate.h — pieces of the GPU file encoders (csg_encode.hip) that are
// plain sequential arithmetic: run-length tokens of a PNG row, deflate
// length codes, length-limited Huffman code lengths, canonical codes, the
// dynamic-block header, Adler-32 / CRC-32 arithmetic, and the "%.6f" text of
// a float32.  Host + device (__host__ __device__ under hipcc), so a CPU test
// harness can exercise the same functions (tests/test_deflate_host.py).
//
// Formats (what the reference writes, generate_construction_data.py):
//   PNG  cv2.imwrite of the RGB frame :1672-1673 and of the JET depth image
//        :1690-1709 -- RFC 2083 8-bit RGB, filter Sub on every row, one zlib
//        stream (RFC 1950) holding one dynamic-Huffman deflate block (RFC
//        1951) of literals and distance-1 matches (run-length, zlib's Z_RLE
//        strategy), split into IDAT chunks of kIdatBytes.
//   CSV  np.savetxt(depth, fmt="%.6f", delimiter=" ") :1687-1688.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define CSG_HD __host__ __device__ __forceinline__
#else
#define CSG_HD inline
#endif

namespace csg {
namespace dfl {

constexpr int kLitCodes = 286;        // 0..255 literals, 256 end of block, 257..285 match lengths
constexpr int kClCodes = 19;          // code-length alphabet
constexpr int kMaxBits = 15;          // deflate code length limit
constexpr int kMaxClBits = 7;         // code-length code limit
constexpr uint32_t kEob = 256;
constexpr uint32_t kIdatBytes = 2048; // zlib bytes per IDAT chunk (one CRC, one GPU thread per chunk)
constexpr uint32_t kMaxHeaderWords = 160;   // 2 zlib bytes + block header bits (< 4,800 bits)
constexpr uint32_t kAdlerMod = 65521;

// Match length 3..258 -> symbol 257..285, extra-bit count and value (RFC 1951 3.2.5).
CSG_HD void length_code(uint32_t len, uint32_t& sym, uint32_t& nextra, uint32_t& extra) {
  if (len <= 10) {
    sym = 254u + len;
    nextra = 0;
    extra = 0;
  } else if (len == 258) {
    sym = 285;
    nextra = 0;
    extra = 0;
  } else {
    const uint32_t l = len - 3u;                       // 8..254
    const uint32_t nb = 31u - (uint32_t)__builtin_clz(l) - 2u;   // 1..5
    sym = 257u + 4u * nb + 4u + ((l >> nb) - 4u);
    nextra = nb;
    extra = l - ((l >> nb) << nb);
  }
}

// The tokens of one run of `len` equal bytes `b`: one literal, then distance-1
// matches of at most 258 bytes, the last < 3 bytes as literals.  `lit(b)`,
// `match(len)` are called in stream order.
template <class Lit, class Match>
CSG_HD void run_tokens(uint32_t b, uint32_t len, Lit&& lit, Match&& match) {
  lit(b);
  uint32_t rem = len - 1u;
  while (rem >= 3u) {
    const uint32_t l = rem < 258u ? rem : 258u;
    match(l);
    rem -= l;
  }
  while (rem--) lit(b);
}

// Streaming run detector over a byte sequence: push() bytes, finish() once.
template <class Lit, class Match>
struct RunTokenizer {
  Lit lit;
  Match match;
  uint32_t rb = 0, rl = 0;
  CSG_HD void push(uint32_t x) {
    if (rl && x == rb) {
      ++rl;
    } else {
      if (rl) run_tokens(rb, rl, lit, match);
      rb = x;
      rl = 1;
    }
  }
  CSG_HD void finish() {
    if (rl) run_tokens(rb, rl, lit, match);
    rl = 0;
  }
};

// Minimum-redundancy code lengths in place (Moffat & Katajainen, "In-place
// calculation of minimum-redundancy codes", 1995): a[0..n) holds weights in
// ascending order on entry and the code length of each on exit
// (non-increasing).  n >= 2.
CSG_HD void mr_lengths(uint32_t* a, int n) {
  a[0] += a[1];
  int root = 0, leaf = 2;
  for (int next = 1; next < n - 1; ++next) {
    if (leaf >= n || a[root] < a[leaf]) {
      a[next] = a[root];
      a[root++] = (uint32_t)next;
    } else {
      a[next] = a[leaf++];
    }
    if (leaf >= n || (root < next && a[root] < a[leaf])) {
      a[next] += a[root];
      a[root++] = (uint32_t)next;
    } else {
      a[next] += a[leaf++];
    }
  }
  a[n - 2] = 0;
  for (int next = n - 3; next >= 0; --next) a[next] = a[a[next]] + 1u;
  int avail = 1, used = 0, depth = 0, root2 = n - 2, next = n - 1;
  while (avail > 0) {
    while (root2 >= 0 && (int)a[root2] == depth) {
      ++used;
      --root2;
    }
    while (avail > used) {
      a[next--] = (uint32_t)depth;
      --avail;
    }
    avail = 2 * used;
    ++depth;
    used = 0;
  }
}

// Length-limited code lengths for the m used symbols `sym[0..m)`, listed in
// ascending (frequency, symbol) order, with frequencies `freq[]`; `w` is
// scratch of m entries; lengths go to len[sym[i]] (unused symbols keep the
// caller's zeros).  The lengths of an optimal code, then the overflow above
// `maxbits` folded back the usual way (each step removes one code at the
// limit and splits one shorter code), and reassigned longest-first to the
// least frequent symbols.  m == 1 gets one code of length 1 (the caller adds
// a second one where the format needs a complete code).
CSG_HD void huff_lengths(const uint32_t* freq, const uint16_t* sym, int m, int maxbits, uint8_t* len, uint32_t* w) {
  if (m <= 0) return;
  if (m == 1) {
    len[sym[0]] = 1;
    return;
  }
  for (int i = 0; i < m; ++i) w[i] = freq[sym[i]];
  mr_lengths(w, m);
  uint32_t cnt[33] = {0};
  for (int i = 0; i < m; ++i) ++cnt[w[i] < 32u ? w[i] : 32u];
  for (int l = maxbits + 1; l <= 32; ++l) {
    cnt[maxbits] += cnt[l];
    cnt[l] = 0;
  }
  uint64_t total = 0;
  for (int l = 1; l <= maxbits; ++l) total += (uint64_t)cnt[l] << (maxbits - l);
  while (total > (1ull << maxbits)) {
    --cnt[maxbits];
    for (int l = maxbits - 1; l > 0; --l) {
      if (cnt[l]) {
        --cnt[l];
        cnt[l + 1] += 2;
        break;
      }
    }
    --total;
  }
  int i = 0;
  for (int l = maxbits; l >= 1; --l)
    for (uint32_t k = 0; k < cnt[l]; ++k) len[sym[i++]] = (uint8_t)l;
}

// Canonical codes (RFC 1951 3.2.2), bit-reversed for LSB-first output:
// code[s] = reversed code | length << 16.
CSG_HD void canonical_codes(const uint8_t* len, int n, uint32_t* code) {
  uint32_t bl[kMaxBits + 1] = {0}, next[kMaxBits + 2] = {0};
  for (int s = 0; s < n; ++s) ++bl[len[s]];
  bl[0] = 0;
  uint32_t c = 0;
  for (int b = 1; b <= kMaxBits; ++b) {
    c = (c + bl[b - 1]) << 1;
    next[b] = c;
  }
  for (int s = 0; s < n; ++s) {
    const uint32_t l = len[s];
    if (!l) {
      code[s] = 0;
      continue;
    }
    uint32_t v = next[l]++, r = 0;
    for (uint32_t k = 0; k < l; ++k) r |= ((v >> k) & 1u) << (l - 1u - k);
    code[s] = r | (l << 16);
  }
}

// LSB-first bit writer into a word array (the dynamic-block header).
struct BitBuf {
  uint32_t* w;
  uint32_t nbits;
  CSG_HD void put(uint32_t v, uint32_t n) {   // n <= 16
    if (!n) return;
    const uint32_t i = nbits >> 5, o = nbits & 31u;
    w[i] |= v << o;
    if (o + n > 32u) w[i + 1] = v >> (32u - o);
    else if (o + n == 32u) w[i + 1] = 0;
    nbits += n;
  }
};

// Order of the code-length code lengths in the header (RFC 1951 3.2.7).
CSG_HD uint32_t cl_order(int i) {
  const uint8_t o[kClCodes] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
  return o[i];
}

// Run-length tokens of the code-length sequence: value | extra << 8 (values
// 0..15 literal lengths, 16 repeat previous 3-6, 17 zeros 3-10, 18 zeros
// 11-138).  Returns the token count (<= n).
CSG_HD int cl_tokens(const uint8_t* lens, int n, uint16_t* tok) {
  int t = 0;
  for (int i = 0; i < n;) {
    const uint32_t v = lens[i];
    int run = 1;
    while (i + run < n && lens[i + run] == v) ++run;
    i += run;
    if (v == 0) {
      while (run >= 11) {
        const int r = run < 138 ? run : 138;
        tok[t++] = (uint16_t)(18u | ((uint32_t)(r - 11) << 8));
        run -= r;
      }
      if (run >= 3) {
        tok[t++] = (uint16_t)(17u | ((uint32_t)(run - 3) << 8));
        run = 0;
      }
      while (run-- > 0) tok[t++] = 0;
    } else {
      tok[t++] = (uint16_t)v;
      --run;
      while (run >= 3) {
        const int r = run < 6 ? run : 6;
        tok[t++] = (uint16_t)(16u | ((uint32_t)(r - 3) << 8));
        run -= r;
      }
      while (run-- > 0) tok[t++] = (uint16_t)v;
    }
  }
  return t;
}

CSG_HD uint32_t cl_extra_bits(uint32_t sym) { return sym == 16 ? 2u : sym == 17 ? 3u : sym == 18 ? 7u : 0u; }

// Adler-32 of the concatenation A | B from (a, b) sums of each part taken
// with a starting value of 0 (a = sum of bytes, b = sum of the running sums),
// all mod 65521; `lenB` = bytes of B.
CSG_HD void adler_cat(uint32_t& a, uint32_t& b, uint32_t a2, uint32_t b2, uint64_t len2) {
  b = (uint32_t)((b + b2 + (uint64_t)(len2 % kAdlerMod) * a) % kAdlerMod);
  a = (a + a2) % kAdlerMod;
}

// CRC-32 (PNG / zlib polynomial, reflected) table entry k.
CSG_HD uint32_t crc_entry(uint32_t k) {
  uint32_t c = k;
  for (int j = 0; j < 8; ++j) c = (c & 1u) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
  return c;
}

// ---------------------------------------------------------------------------
// "%.6f" of a float32, byte-identical to np.savetxt's "%.6f" % float(x):
// x * 10^6 rounded half to even from the exact binary value; "inf", "-inf",
// "nan".  Writes at most kMaxF6Chars bytes to out, returns the count.
// ---------------------------------------------------------------------------
constexpr int kMaxF6Chars = 48;

CSG_HD int dec_digits_u32(uint32_t v) {
  int n = 1;
  while (v >= 10u) {
    v /= 10u;
    ++n;
  }
  return n;
}

CSG_HD int dec_digits_u64(uint64_t v) {
  int n = 1;
  while (v >= 10u) {
    v /= 10u;
    ++n;
  }
  return n;
}

// Digits written from the last one backwards straight into `out` (no local
// array: on the GPU a dynamically indexed one lives in scratch memory).
CSG_HD int put_dec_u64(char* out, uint64_t v) {
  const int n = dec_digits_u64(v);
  for (int k = n - 1; k >= 0; --k) {
    out[k] = (char)('0' + v % 10u);
    v /= 10u;
  }
  return n;
}

CSG_HD int put_dec_u32(char* out, uint32_t v) {
  const int n = dec_digits_u32(v);
  for (int k = n - 1; k >= 0; --k) {
    out[k] = (char)('0' + v % 10u);
    v /= 10u;
  }
  return n;
}

// x * 10^6 rounded half to even, for x = m * 2^e (m < 2^24, e < 17).
CSG_HD uint64_t scaled6(uint64_t m, int e) {
  if (e >= 0) return (m << e) * 1000000u;   // m << e < 2^41: fits
  const uint64_t n = m * 1000000u;          // < 2^44
  const int sh = -e;
  if (sh >= 64) return 0;
  uint64_t q = n >> sh;
  const uint64_t r = n & ((1ull << sh) - 1u), half = 1ull << (sh - 1);
  if (r > half || (r == half && (q & 1u))) ++q;
  return q;
}

CSG_HD int fmt6f(float x, char* out) {
  uint32_t u;
  __builtin_memcpy(&u, &x, 4);
  const uint32_t ex = (u >> 23) & 255u, mant = u & 0x7FFFFFu;
  int p = 0;
  if (ex == 255u) {
    if (mant) {
      out[0] = 'n'; out[1] = 'a'; out[2] = 'n';
      return 3;
    }
    if (u >> 31) out[p++] = '-';
    out[p++] = 'i'; out[p++] = 'n'; out[p++] = 'f';
    return p;
  }
  if (u >> 31) out[p++] = '-';
  const uint64_t m = ex ? (mant | 0x800000u) : mant;
  const int e = ex ? (int)ex - 150 : -149;
  if (e >= 17) {
    // an integer of up to 128 bits (m * 2^e): decimal digits by long division
    // of 32-bit limbs by 10^9, then ".000000"
    uint32_t limb[4] = {0, 0, 0, 0};
    const int w = e >> 5, b = e & 31;
    const uint64_t sh = m << b;   // < 2^55
    limb[w] = (uint32_t)sh;
    if (w + 1 < 4) limb[w + 1] = (uint32_t)(sh >> 32);
    uint32_t chunks[5];
    int nc = 0;
    for (;;) {
      bool zero = true;
      uint64_t r = 0;
      for (int k = 3; k >= 0; --k) {
        const uint64_t cur = (r << 32) | limb[k];
        limb[k] = (uint32_t)(cur / 1000000000u);
        r = cur % 1000000000u;
        zero &= limb[k] == 0;
      }
      chunks[nc++] = (uint32_t)r;
      if (zero) break;
    }
    p += put_dec_u64(out + p, chunks[nc - 1]);
    for (int k = nc - 2; k >= 0; --k) {
      uint32_t c = chunks[k];
      for (int d = 8; d >= 0; --d) {
        out[p + d] = (char)('0' + c % 10u);
        c /= 10u;
      }
      p += 9;
    }
    out[p++] = '.';
    for (int d = 0; d < 6; ++d) out[p++] = '0';
    return p;
  }
  const uint64_t q = scaled6(m, e);
  if (q < (1ull << 32)) {   // |x| < ~4295 (depths): 32-bit digit arithmetic
    const uint32_t q32 = (uint32_t)q, ip = q32 / 1000000u;
    uint32_t f = q32 - ip * 1000000u;
    p += put_dec_u32(out + p, ip);
    out[p++] = '.';
    for (int d = 5; d >= 0; --d) {
      out[p + d] = (char)('0' + f % 10u);
      f /= 10u;
    }
    return p + 6;
  }
  const uint64_t ip = q / 1000000u;
  uint32_t f = (uint32_t)(q - ip * 1000000u);
  p += put_dec_u64(out + p, ip);
  out[p++] = '.';
  for (int d = 5; d >= 0; --d) {
    out[p + d] = (char)('0' + f % 10u);
    f /= 10u;
  }
  return p + 6;
}

// Length of fmt6f(x) without writing it.
CSG_HD int fmt6f_len(float x) {
  uint32_t u;
  __builtin_memcpy(&u, &x, 4);
  const uint32_t ex = (u >> 23) & 255u, mant = u & 0x7FFFFFu;
  const int sign = (int)(u >> 31);
  if (ex == 255u) return mant ? 3 : 3 + sign;
  const uint64_t m = ex ? (mant | 0x800000u) : mant;
  const int e = ex ? (int)ex - 150 : -149;
  if (e >= 17) {
    char tmp[kMaxF6Chars];
    return fmt6f(x, tmp);
  }
  const uint64_t q = scaled6(m, e);
  if (q < (1ull << 32)) return sign + dec_digits_u32((uint32_t)q / 1000000u) + 7;
  return sign + dec_digits_u64(q / 1000000u) + 7;
}

// "%.6f" of an integer 0..255 (a point's colour channel as np.savetxt prints
// it after np.hstack promotes it to float): its digits, then ".000000".
CSG_HD int fmt6f_u8_len(uint32_t v) { return (v >= 100u ? 3 : v >= 10u ? 2 : 1) + 7; }
CSG_HD int fmt6f_u8(uint32_t v, char* out) {
  const int n = put_dec_u32(out, v);
  out[n] = '.';
  for (int d = 1; d <= 6; ++d) out[n + d] = '0';
  return n + 7;
}

// One point-cloud line "x y z r g b\n" (np.savetxt(np.hstack([xyz, rgb]),
// fmt="%.6f", delimiter=" "), GDP:766-770): its length, and its text.
constexpr int kMaxPcdLine = 3 * kMaxF6Chars + 3 * 10 + 6;
CSG_HD int pcd_line_len(float x, float y, float z, uint32_t r, uint32_t g, uint32_t b) {
  return fmt6f_len(x) + fmt6f_len(y) + fmt6f_len(z) + fmt6f_u8_len(r) + fmt6f_u8_len(g) + fmt6f_u8_len(b) + 6;
}
CSG_HD int pcd_line(float x, float y, float z, uint32_t r, uint32_t g, uint32_t b, char* out) {
  int p = fmt6f(x, out);
  out[p++] = ' ';
  p += fmt6f(y, out + p);
  out[p++] = ' ';
  p += fmt6f(z, out + p);
  out[p++] = ' ';
  p += fmt6f_u8(r, out + p);
  out[p++] = ' ';
  p += fmt6f_u8(g, out + p);
  out[p++] = ' ';
  p += fmt6f_u8(b, out + p);
  out[p++] = '\n';
  return p;
}
// The file's first line (header="x y z r g b", comments="").
constexpr uint32_t kPcdHeaderBytes = 12;
CSG_HD char pcd_header_byte(uint32_t k) { return "x y z r g b\n"[k]; }
// A pixel is a point when its world position is a number (NaN: nothing hit).
CSG_HD bool pcd_valid(float x, float y, float z) { return x == x && y == y && z == z; }

}  // namespace dfl
}  // namespace csg
