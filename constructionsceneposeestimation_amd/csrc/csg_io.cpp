// libcsgio.so: host-side writers of the generator's on-disk formats
// (include/csg_io.h).  Each call writes one file; no shared state, so the
// Python generator runs a pool of threads through ctypes (which releases the
// GIL) while the GPU renders the next batch.
#include "../../include/csg_io.h"

#include "csg_repr.h"

#include <zlib.h>

#include <cerrno>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace {

struct File {
  FILE* f = nullptr;
  explicit File(const char* path) : f(path ? std::fopen(path, "wb") : nullptr) {}
  ~File() {
    if (f) std::fclose(f);
  }
  bool write(const void* p, size_t n) { return std::fwrite(p, 1, n, f) == n; }
  int close() {
    const int rc = std::fclose(f);
    f = nullptr;
    return rc == 0 ? 0 : -EIO;
  }
};

void put_be32(std::vector<uint8_t>& v, uint32_t x) {
  v.push_back((uint8_t)(x >> 24));
  v.push_back((uint8_t)(x >> 16));
  v.push_back((uint8_t)(x >> 8));
  v.push_back((uint8_t)x);
}

void png_chunk(std::vector<uint8_t>& out, const char* type, const uint8_t* data, size_t n) {
  put_be32(out, (uint32_t)n);
  const size_t at = out.size();
  out.insert(out.end(), type, type + 4);
  if (n) out.insert(out.end(), data, data + n);
  const uint32_t crc = (uint32_t)crc32(0L, out.data() + at, (uInt)(n + 4));
  put_be32(out, crc);
}

// "%.6f" of a double, as Python's % operator formats it for np.savetxt
// (std::to_chars is correctly rounded, ties to even, like Python's dtoa;
// NaN prints as "nan" whatever its sign bit, as Python does).
inline char* fmt6(char* p, char* end, double x) {
  if (std::isnan(x)) {
    std::memcpy(p, "nan", 3);
    return p + 3;
  }
  return std::to_chars(p, end, x, std::chars_format::fixed, 6).ptr;
}

// "00" "01" ... "99"
constexpr char kDigits2[201] =
    "00010203040506070809101112131415161718192021222324252627282930313233343536373839"
    "40414243444546474849505152535455565758596061626364656667686970717273747576777879"
    "8081828384858687888990919293949596979899";

// Decimal digits of v (v < 10^20), most significant first.
inline char* put_u64(char* p, uint64_t v) {
  char tmp[20];
  int n = 0;
  do {
    tmp[n++] = (char)('0' + v % 10u);
    v /= 10u;
  } while (v);
  while (n) *p++ = tmp[--n];
  return p;
}

// "%.6f" of a float32 value, exactly as fmt6 of its double: the value is
// m * 2^e with a 24-bit m, so x * 10^6 = m * 10^6 * 2^e is an integer (m *
// 10^6 < 2^44) shifted right by -e, rounded half to even from the exact
// remainder -- no floating point, about 4x faster than to_chars.  Values of
// 2^40 and above take fmt6.
inline char* fmt6f(char* p, char* end, float x) {
  uint32_t u;
  std::memcpy(&u, &x, 4);
  const uint32_t ex = (u >> 23) & 255u, mant = u & 0x7FFFFFu;
  if (ex == 255u || ex >= 127u + 40u) return fmt6(p, end, (double)x);   // inf, nan, huge
  const uint64_t m = ex ? (mant | 0x800000u) : mant;
  const int e = ex ? (int)ex - 150 : -149;
  if (u >> 31) *p++ = '-';
  uint64_t q;
  if (e >= 0) {
    q = (m << e) * 1000000u;   // an integer: < 2^64 / 10^6 here
  } else {
    const uint64_t n = m * 1000000u;
    const int sh = -e;
    if (sh >= 64) {
      q = 0;                   // n < 2^44 <= half
    } else {
      q = n >> sh;
      const uint64_t r = n & ((1ull << sh) - 1u), half = 1ull << (sh - 1);
      if (r > half || (r == half && (q & 1u))) ++q;
    }
  }
  const uint64_t ip = q / 1000000u;
  const uint32_t f = (uint32_t)(q - ip * 1000000u);
  if (ip < 10u) {
    *p++ = (char)('0' + ip);
  } else if (ip < 100u) {
    std::memcpy(p, kDigits2 + 2 * ip, 2);
    p += 2;
  } else if (ip < 1000u) {
    *p++ = (char)('0' + ip / 100u);
    std::memcpy(p, kDigits2 + 2 * (ip % 100u), 2);
    p += 2;
  } else {
    p = put_u64(p, ip);
  }
  *p++ = '.';
  std::memcpy(p, kDigits2 + 2 * (f / 10000u), 2);
  std::memcpy(p + 2, kDigits2 + 2 * ((f / 100u) % 100u), 2);
  std::memcpy(p + 4, kDigits2 + 2 * (f % 100u), 2);
  return p + 6;
}

}  // namespace

extern "C" {

int csgio_abi_version(void) { return CSGIO_ABI_VERSION; }

int csgio_write_png_rgb(const char* path, const uint8_t* rgb, uint32_t w, uint32_t h, int level, int strategy) {
  if (!path || !rgb || !w || !h || level < 0 || level > 9 || strategy < 0 || strategy > 2) return -EINVAL;
  // filter type 1 (Sub) on every row: byte minus the byte one pixel to the left
  const size_t stride = (size_t)w * 3;
  std::vector<uint8_t> raw((stride + 1) * h);
  for (uint32_t y = 0; y < h; ++y) {
    uint8_t* d = &raw[(stride + 1) * y];
    const uint8_t* s = rgb + stride * y;
    d[0] = 1;
    std::memcpy(d + 1, s, 3);
    for (size_t x = 3; x < stride; ++x) d[1 + x] = (uint8_t)(s[x] - s[x - 3]);
  }
  uLongf zn = compressBound((uLong)raw.size());
  std::vector<uint8_t> z(zn);
  {
    z_stream zs{};
    static const int kStrategy[3] = {Z_DEFAULT_STRATEGY, Z_RLE, Z_HUFFMAN_ONLY};
    if (deflateInit2(&zs, level, Z_DEFLATED, 15, 9, kStrategy[strategy]) != Z_OK) return -EIO;
    zs.next_in = raw.data();
    zs.avail_in = (uInt)raw.size();
    zs.next_out = z.data();
    zs.avail_out = (uInt)zn;
    const int rc = deflate(&zs, Z_FINISH);
    zn = zs.total_out;
    deflateEnd(&zs);
    if (rc != Z_STREAM_END) return -EIO;
  }
  std::vector<uint8_t> out;
  out.reserve(zn + 64);
  static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
  out.insert(out.end(), sig, sig + 8);
  std::vector<uint8_t> ihdr;
  put_be32(ihdr, w);
  put_be32(ihdr, h);
  ihdr.push_back(8);   // bit depth
  ihdr.push_back(2);   // colour type RGB
  ihdr.push_back(0);   // deflate
  ihdr.push_back(0);   // adaptive filtering
  ihdr.push_back(0);   // no interlace
  png_chunk(out, "IHDR", ihdr.data(), ihdr.size());
  png_chunk(out, "IDAT", z.data(), zn);
  png_chunk(out, "IEND", nullptr, 0);
  File f(path);
  if (!f.f) return -errno;
  if (!f.write(out.data(), out.size())) return -EIO;
  return f.close();
}

int csgio_write_npy(const char* path, const void* data, uint64_t nbytes, const char* descr, const uint64_t* shape,
                    uint32_t ndim) {
  if (!path || (!data && nbytes) || !descr || (!shape && ndim)) return -EINVAL;
  std::string dict = std::string("{'descr': '") + descr + "', 'fortran_order': False, 'shape': (";
  for (uint32_t k = 0; k < ndim; ++k) {
    dict += std::to_string(shape[k]);
    if (ndim == 1 || k + 1 < ndim) dict += ",";
    if (k + 1 < ndim) dict += " ";
  }
  dict += "), }";
  // magic(6) + version(2) + header length(2) + dict + padding + '\n', total % 64 == 0
  size_t total = 10 + dict.size() + 1;
  const size_t pad = (64 - total % 64) % 64;
  dict.append(pad, ' ');
  dict += '\n';
  const uint16_t hl = (uint16_t)dict.size();
  File f(path);
  if (!f.f) return -errno;
  const uint8_t head[8] = {0x93, 'N', 'U', 'M', 'P', 'Y', 1, 0};
  const uint8_t hlb[2] = {(uint8_t)(hl & 255u), (uint8_t)(hl >> 8)};
  if (!f.write(head, 8) || !f.write(hlb, 2) || !f.write(dict.data(), dict.size())) return -EIO;
  if (nbytes && !f.write(data, nbytes)) return -EIO;
  return f.close();
}

int csgio_write_depth_csv(const char* path, const float* d, uint32_t w, uint32_t h) {
  if (!path || !d || !w || !h) return -EINVAL;
  File f(path);
  if (!f.f) return -errno;
  std::vector<char> line((size_t)w * 48 + 2);
  for (uint32_t y = 0; y < h; ++y) {
    char* p = line.data();
    char* end = line.data() + line.size();
    for (uint32_t x = 0; x < w; ++x) {
      if (x) *p++ = ' ';
      p = fmt6f(p, end, d[(size_t)y * w + x]);
    }
    *p++ = '\n';
    if (!f.write(line.data(), (size_t)(p - line.data()))) return -EIO;
  }
  return f.close();
}

int csgio_depth_stats(const float* d, uint64_t n, double* out) {
  if ((!d && n) || !out) return -EINVAL;
  uint64_t valid = 0, zero = 0, inf = 0;
  double sum = 0.0;
  float lo = INFINITY, hi = -INFINITY;
  for (uint64_t k = 0; k < n; ++k) {
    const float v = d[k];
    if (v > 0.0f && v < INFINITY) {
      ++valid;
      sum += (double)v;
      lo = v < lo ? v : lo;
      hi = v > hi ? v : hi;
    } else if (v == 0.0f) {
      ++zero;
    } else if (std::isinf(v)) {
      ++inf;
    }
  }
  out[0] = (double)valid;
  out[1] = (double)zero;
  out[2] = (double)inf;
  out[3] = sum;
  out[4] = valid ? (double)lo : 0.0;
  out[5] = valid ? (double)hi : 0.0;
  return 0;
}

int csgio_write_pointcloud_txt(const char* path, const float* xyz, const uint8_t* rgb, uint64_t n) {
  if (!path || (n && (!xyz || !rgb))) return -EINVAL;
  File f(path);
  if (!f.f) return -errno;
  static const char head[] = "x y z r g b\n";
  if (!f.write(head, sizeof(head) - 1)) return -EIO;
  std::vector<char> buf(1 << 20);
  size_t used = 0;
  for (uint64_t k = 0; k < n; ++k) {
    const float* p3 = xyz + 3 * k;
    if (std::isnan(p3[0]) || std::isnan(p3[1]) || std::isnan(p3[2])) continue;
    if (buf.size() - used < 6 * 48 + 2) {
      if (!f.write(buf.data(), used)) return -EIO;
      used = 0;
    }
    char* p = buf.data() + used;
    char* end = buf.data() + buf.size();
    for (int c = 0; c < 3; ++c) {
      p = fmt6f(p, end, p3[c]);
      *p++ = ' ';
    }
    for (int c = 0; c < 3; ++c) {
      p = put_u64(p, rgb[3 * k + c]);   // "%.6f" of an integer
      std::memcpy(p, ".000000", 7);
      p += 7;
      *p++ = c < 2 ? ' ' : '\n';
    }
    used = (size_t)(p - buf.data());
  }
  if (used && !f.write(buf.data(), used)) return -EIO;
  return f.close();
}

int csgio_write_label_json(const char* path, const csgio_label* L) {
  if (!path || !L || !L->camera_pose || !L->camera_params || !L->class_mapping || (L->n_objects && (!L->obj_head ||
      !L->obj_label || !L->obj_kp_off)) || (L->n_labels && !L->inst_stats) || (L->n_kp && (!L->kp_uv || !L->kp_vis ||
      !L->kp_name)))
    return -EINVAL;
  std::string o;
  o.reserve(131072);
  char num[48];
  auto put_int = [&](long long v) { o.append(num, std::to_chars(num, num + sizeof num, v).ptr); };
  auto put_dbl = [&](double v) {
    if (std::isnan(v)) o += "NaN";
    else if (std::isinf(v)) o += v > 0 ? "Infinity" : "-Infinity";
    else o.append(num, csg::repr_double(num, v));
  };
  o += "{\n  \"frame_id\": ";
  put_int(L->frame_id);
  o += ",\n  \"camera_pose\": [";
  for (int k = 0; k < 7; ++k) {
    o += k ? ",\n    " : "\n    ";
    put_dbl(L->camera_pose[k]);
  }
  o += "\n  ],\n  \"camera_params\": ";
  o += L->camera_params;
  o += ",\n  \"objects\": ";
  uint32_t n_vis = 0;
  for (uint32_t j = 0; j < L->n_objects; ++j) {
    const int32_t lab = L->obj_label[j];
    if (lab < 0 || (uint32_t)lab >= L->n_labels) continue;
    const uint32_t* st = L->inst_stats + (size_t)lab * 5;
    const bool hidden = st[0] == 0;
    if (hidden && !(L->obj_listed && L->obj_listed[j])) continue;
    o += n_vis++ ? ",\n    {\n" : "[\n    {\n";
    o += L->obj_head[j];
    o += ",\n      \"pixel_count\": ";
    put_int(st[0]);
    o += ",\n      \"bbox_2d\": [";
    for (int k = 1; k < 5; ++k) {
      o += k > 1 ? ",\n        " : "\n        ";
      put_int(hidden ? -1 : (long long)st[k]);
    }
    o += "\n      ]";
    if (L->covered) {   // occlusionRatio: 1 - visible / covered, float32 (labels.occlusion_ratios); -1 unknown
      const uint32_t cv = L->covered[lab];
      const uint32_t cnt = cv & 0x7FFFFFFFu;
      const bool known = !(cv & 0x80000000u);
      const float occ = hidden ? (known ? 1.0f : -1.0f)
                               : (known && cnt) ? (float)(1.0 - (double)st[0] / (double)cnt) : -1.0f;
      o += ",\n      \"occlusion_ratio\": ";
      put_dbl((double)occ);
    }
    const uint32_t k0 = L->obj_kp_off[j], k1 = L->obj_kp_off[j + 1];
    if (k1 > k0) {
      o += ",\n      \"keypoints_2d\": [";
      for (uint32_t q = k0; q < k1; ++q) {
        const uint32_t k = L->obj_kp[q];
        o += q > k0 ? ",\n        [\n          " : "\n        [\n          ";
        o += L->kp_name[k];
        o += ",\n          ";
        put_dbl((double)L->kp_uv[2 * k]);
        o += ",\n          ";
        put_dbl((double)L->kp_uv[2 * k + 1]);
        o += ",\n          ";
        put_int(L->kp_vis[k]);
        o += "\n        ]";
      }
      o += "\n      ]";
    }
    o += "\n    }";
  }
  o += n_vis ? "\n  ]" : "[]";
  o += ",\n  \"instance_mask_shape\": [\n    ";
  put_int(L->height);
  o += ",\n    ";
  put_int(L->width);
  o += "\n  ],\n  \"num_objects\": ";
  put_int(n_vis);
  o += ",\n  \"class_mapping\": ";
  o += L->class_mapping;
  o += "\n}";
  File f(path);
  if (!f.f) return -errno;
  if (!f.write(o.data(), o.size())) return -EIO;
  return f.close();
}

}  // extern "C"
