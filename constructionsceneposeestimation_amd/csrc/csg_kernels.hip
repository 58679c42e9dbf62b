// gfx950 (MI355X / CDNA4) kernels of the construction-scene frame generator.
//
// Replaces the per-frame render + annotate step the reference gets from
// Isaac Sim RTX + Replicator (generate_construction_data.py:1586-1595 pose +
// render, :1669 RGB, :1681 depth, :1475/:1909 instance mask, :1780/:1916
// bounding boxes).  The arithmetic follows DESIGN.md "Raster spec" exactly:
// this file must stay bit-identical to oracle/csg_oracle.c (built with
// -ffp-contract=off on both sides; every float expression below is written
// in the same order as there).
//
// Pipeline per launch chain of F frames (by default the whole batch):
//   k_clip     (instances x F)   P*V*M in fp32, fixed summation order
//   k_setup    (F x chunks)      chunk AABB cull, transform, triangle cull,
//                                near-clip, fixed-point setup, exact cover
//                                test of small records, wave-ballot append
//   k_count    (128 x F)         LDS-aggregated per-tile record counts
//   k_scan     (F)               exclusive scan of tile counts
//   k_bin      (128 x F)         LDS-aggregated scatter of record ids to bins
//   k_keypoints(K x F)           3D->2D keypoint projection (before k_raster;
//                                k_raster depth-tests those in its tile)
//   k_raster   (tiles x F)       32x32 tile: bins staged in LDS, (record,row)
//                                then (span,pixel) expansion, 64-bit
//                                (depth,uid) z-buffer in LDS (ds_min_u64),
//                                then resolve: texture, shade, instance id,
//                                optional depth / normals / points / label
//                                stats, coalesced HBM writes
// The kernels are VALU-issue bound: the code below trades
// memory for instructions wherever the result is unchanged.
#include <math.h>

#include <algorithm>

#include <type_traits>

#include "csg_kernels.h"

namespace csg {

#ifndef CSG_ABLATION
#define CSG_ABLATION 0         // 1: honour the CSG_DEBUG ablation / profiling bits (tools/ablate.sh builds)
#endif
#define DBG(d) (CSG_ABLATION ? (d) : 0u)
// Every code path below is the production one (measured alternatives are in
// DESIGN.md §6 "Measured and rejected"; tools/build_variant.sh rebuilds old
// revisions for A/B).  The remaining macros are tuning constants of the same
// code (CSG_STAGE, CSG_WAVES, ...), not alternative paths.

constexpr int kSmallCover = 4;   // records with at most 4 x 4 pixel centres get an exact cover test in k_setup
constexpr uint64_t kEmptyKey = ~0ull;
constexpr float kGuardPx = 1048576.0f;

// ---------------------------------------------------------------------------
// shared arithmetic (mirrors csg_oracle.c line by line)
// ---------------------------------------------------------------------------
typedef float f32x2 __attribute__((ext_vector_type(2)));   // packed FP32 pair (v_pk_*_f32)

__device__ __forceinline__ float dot4(const float* r, float x, float y, float z) {
  return ((r[0] * x + r[1] * y) + r[2] * z) + r[3];
}

__device__ __forceinline__ void mat4_mul(const float* a, const float* b, float* c) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      c[i * 4 + j] = ((a[i * 4 + 0] * b[0 * 4 + j] + a[i * 4 + 1] * b[1 * 4 + j]) + a[i * 4 + 2] * b[2 * 4 + j]) +
                     a[i * 4 + 3] * b[3 * 4 + j];
}

// 1.0f / x, bit-identical to the IEEE division for |x| in [2^-126, 2^126]:
// the hardware reciprocal (~1 ulp) plus one Newton step with an exact FMA
// residual, 3 VALU instead of the division's 11 (v_div_scale x2, v_rcp, 6 FMAs,
// v_div_fmas, v_div_fixup).  Checked exhaustively on the MI355X over every
// normal float of both signs (tools/rcp_check.hip, profiles/r04/rcp_check.json):
// the only differences are the 2 x (2^24 - 1) x with |x| > 2^126, whose
// reciprocal is subnormal.  k_raster's inverse depths lie in [1/far, 1/near],
// inside the range (csg_create keeps near / far clip in [2^-126, 2^126]).
// k_setup uses it for the per-vertex 1/W (W >= near_clip after near-plane
// clipping; setup -1.9%, profiles/r04/ab/setup_w_rcp.txt) and, range-checked,
// for 1/det (hom_setup: -0.5%, profiles/r04/ab/det_rcp.txt); the near-plane
// crossing is a true quotient and stays a division.  (Round 4's first
// attempt, every k_setup division range-checked at once, measured 3% slower:
// profiles/r04/ab/rcp_packed_smallcover.txt.)  CSG_FAST_RCP=0 builds the
// division (A/B).
#ifndef CSG_FAST_RCP
#define CSG_FAST_RCP 1
#endif
__device__ __forceinline__ float rcp_ieee(float x) {
#if CSG_FAST_RCP
  const float r0 = __builtin_amdgcn_rcpf(x);
  const float e = __builtin_fmaf(-x, r0, 1.0f);
  return __builtin_fmaf(e, r0, r0);
#else
  return 1.0f / x;
#endif
}

struct Cv3 { float x, y, w; };

struct Hom {
  float A[3], B[3], C[3];
  float invdet;
  bool ok;
};

__device__ __forceinline__ void hom_setup(const Cv3* v, Hom& h) {
  const int ea[3] = {1, 2, 0}, eb[3] = {2, 0, 1};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const Cv3 a = v[ea[k]], b = v[eb[k]];
    h.A[k] = a.y * b.w - a.w * b.y;
    h.B[k] = a.w * b.x - a.x * b.w;
    h.C[k] = a.x * b.y - a.y * b.x;
  }
  const float det = (v[0].x * h.A[0] + v[0].y * h.B[0]) + v[0].w * h.C[0];
  h.ok = det != 0.0f;
  // 1/det: the Newton reciprocal inside its proven range, the division outside
  const float ad = fabsf(det);
  h.invdet = !h.ok ? 0.0f : (ad >= 0x1p-126f && ad <= 0x1p126f) ? rcp_ieee(det) : 1.0f / det;
}

// Screen-space planes of the original triangle (spec §3.5-6), from its
// homogeneous edge rows: with e_k = A_k*x + B_k*y + C_k, 1/W = invdet * sum e_k
// and u/W = invdet * sum e_k u_k are affine in (x, y):
//   D = (((A0 + A1) + A2) * invdet, (B...) * invdet, (C...) * invdet)
//   U = (((A0*u0 + A1*u1) + A2*u2) * invdet, ...), V likewise with v.
// uv = u0 v0 u1 v1 u2 v2.
__device__ __forceinline__ void depth_plane(const float* A, const float* B, const float* C, float invdet, float* D) {
  D[0] = ((A[0] + A[1]) + A[2]) * invdet;
  D[1] = ((B[0] + B[1]) + B[2]) * invdet;
  D[2] = ((C[0] + C[1]) + C[2]) * invdet;
}
__device__ __forceinline__ void uv_planes(const float* A, const float* B, const float* C, float invdet,
                                          const float* uv, float* U, float* V) {
  U[0] = ((A[0] * uv[0] + A[1] * uv[2]) + A[2] * uv[4]) * invdet;
  U[1] = ((B[0] * uv[0] + B[1] * uv[2]) + B[2] * uv[4]) * invdet;
  U[2] = ((C[0] * uv[0] + C[1] * uv[2]) + C[2] * uv[4]) * invdet;
  V[0] = ((A[0] * uv[1] + A[1] * uv[3]) + A[2] * uv[5]) * invdet;
  V[1] = ((B[0] * uv[1] + B[1] * uv[3]) + B[2] * uv[5]) * invdet;
  V[2] = ((C[0] * uv[1] + C[1] * uv[3]) + C[2] * uv[5]) * invdet;
}

// A plane at pixel centre (fx, fy) = (px + 0.5, py + 0.5).
__device__ __forceinline__ float plane_at(float p0, float p1, float p2, float fx, float fy) {
  return (p0 * fx + p1 * fy) + p2;
}

// Bilinear RGBA8, repeat wrap, 8-bit fixed weights (v flipped: row 0 = top).
struct TexTap { uint32_t i00, i10, i01, i11; int wx, wy; };

// fu mod n in [0, n) for an integer-valued |fu| < 2^23, without an integer
// division: q may be off by one (approximate reciprocal), one correction fixes
// it; q*n and fu - q*n are integers below 2^24, so every step is exact.
__device__ __forceinline__ int wrap_index(float fu, int n) {
  const float nf = (float)n;
  // Texture coordinates inside one repeat (the usual case: uvs in [0, 1])
  // need no reduction; the branch is skipped when no lane of the wave wraps.
  if (fu >= 0.0f && fu < nf) return (int)fu;
  const float q = floorf(fu * __builtin_amdgcn_rcpf(nf));
  float r = fu - q * nf;
  r += r < 0.0f ? nf : 0.0f;
  r -= r >= nf ? nf : 0.0f;
  return (int)r;
}

// Texel coordinates (u * tw - 0.5, (1 - v) * th - 0.5) as one packed multiply and add
__device__ __forceinline__ f32x2 texel_coords(float u, float v, int tw, int th) {
  const f32x2 a = {u, 1.0f - v}, n = {(float)tw, (float)th};
  return a * n - 0.5f;
}

__device__ __forceinline__ TexTap tex_taps(int tw, int th, float u, float v) {   // tw, th <= 16384
  const f32x2 t2 = texel_coords(u, v, tw, th);
  float tu = t2.x, tv = t2.y;
  if (!(fabsf(tu) < 8388608.0f)) tu = 0.0f;
  if (!(fabsf(tv) < 8388608.0f)) tv = 0.0f;
  const float fu = floorf(tu), fv = floorf(tv);
  TexTap t;
  // tu - fu is exact and in [0, 1), so the weights are in [0, 255] and the
  // wrapped indices below 16384 (upload limit): the masks change no value,
  // they let the compiler use full-rate 24-bit multiplies
  t.wx = (int)((tu - fu) * 256.0f) & 255;
  t.wy = (int)((tv - fv) * 256.0f) & 255;
  tw &= 0x7FFF;
  const int x0 = wrap_index(fu, tw) & 0x3FFF, y0 = wrap_index(fv, th) & 0x3FFF;
  const int x1 = (x0 + 1 == tw) ? 0 : x0 + 1;
  const int y1 = (y0 + 1 == th) ? 0 : y0 + 1;
  const uint32_t r0 = __umul24((uint32_t)y0, (uint32_t)tw), r1 = __umul24((uint32_t)y1, (uint32_t)tw);
  t.i00 = r0 + (uint32_t)x0; t.i10 = r0 + (uint32_t)x1;
  t.i01 = r1 + (uint32_t)x0; t.i11 = r1 + (uint32_t)x1;
  return t;
}

// Operands are below 2^24 (channels <= 255, weights <= 256), so every
// product is a full-rate 24-bit multiply (a plain int multiply here becomes
// the quarter-rate v_mul_lo_u32).
__device__ __forceinline__ int bilerp8(uint32_t c00, uint32_t c10, uint32_t c01, uint32_t c11, int wx, int wy) {
  const uint32_t ax = 256u - (uint32_t)wx, ay = 256u - (uint32_t)wy;
  const uint32_t top = __umul24(c00, ax) + __umul24(c10, (uint32_t)wx);
  const uint32_t bot = __umul24(c01, ax) + __umul24(c11, (uint32_t)wx);
  return (int)((__umul24(top, ay) + __umul24(bot, (uint32_t)wy) + 32768u) >> 16);
}

// x / 255 for 0 <= x < 2^16 (exhaustively equal), one 24-bit multiply
__device__ __forceinline__ int div255(uint32_t x) { return (int)(__umul24(x, 32897u) >> 23); }

__device__ __forceinline__ int tex_channel(uint32_t c00, uint32_t c10, uint32_t c01, uint32_t c11, int sh, int wx,
                                           int wy) {
  return bilerp8((c00 >> sh) & 255u, (c10 >> sh) & 255u, (c01 >> sh) & 255u, (c11 >> sh) & 255u, wx, wy);
}

__device__ __forceinline__ void tex_sample(const SceneDev& s, int tid, float u, float v, int out[4]) {
  const TexDesc t = s.texd[tid];
  const TexTap k = tex_taps((int)t.width, (int)t.height, u, v);
  const uint32_t* base = reinterpret_cast<const uint32_t*>(s.texels) + t.offset;
  const uint32_t c00 = base[k.i00], c10 = base[k.i10], c01 = base[k.i01], c11 = base[k.i11];
#pragma unroll
  for (int c = 0; c < 4; ++c) out[c] = tex_channel(c00, c10, c01, c11, 8 * c, k.wx, k.wy);
}

// The alpha test: bilinear alpha (8-bit weights, as tex_sample) > thr.
// The alpha-quad image holds at texel (x, y) the alphas of (x,y), (x+1,y),
// (x,y+1), (x+1,y+1) (wrapped), so the bilinear footprint is one 4-byte load.
// First the 2-bit class of that quad (acls, 16 per word, 1/16 of the quad
// image, so it stays in L2): all four alphas <= thr -> the filtered value is
// too (weights sum to 65536 and the rounding cannot cross an integer), fail;
// all four > thr -> pass; only mixed quads (~5% of a foliage card's texels)
// load the quad and filter.  `wh` = width | height << 16.
__device__ __forceinline__ bool alpha_pass(const uint32_t* aquad, const uint32_t* acls, uint32_t offset, uint32_t wh,
                                           int thr, float u, float v) {
  const int tw = (int)(wh & 0xFFFFu), th = (int)(wh >> 16);
  const f32x2 t2 = texel_coords(u, v, tw, th);
  float tu = t2.x, tv = t2.y;
  if (!(fabsf(tu) < 8388608.0f)) tu = 0.0f;
  if (!(fabsf(tv) < 8388608.0f)) tv = 0.0f;
  const float fu = floorf(tu), fv = floorf(tv);
  const uint32_t idx = offset + __umul24((uint32_t)wrap_index(fv, th) & 0x3FFFu, (uint32_t)tw & 0x7FFFu) +
                       ((uint32_t)wrap_index(fu, tw) & 0x3FFFu);   // (masks: see tex_taps)
  const uint32_t cl = (acls[idx >> 4] >> (2u * (idx & 15u))) & 3u;
  if (cl != 3u) return cl != 0u;
  const int wx = (int)((tu - fu) * 256.0f) & 255, wy = (int)((tv - fv) * 256.0f) & 255;
  const uint32_t q = aquad[idx];
  return bilerp8(q & 255u, (q >> 8) & 255u, (q >> 16) & 255u, q >> 24, wx, wy) > thr;
}

__device__ __forceinline__ uint32_t fbits(float f) { return __float_as_uint(f); }

// ---------------------------------------------------------------------------
// wave / block helpers (wave64)
// ---------------------------------------------------------------------------
// Inclusive wave64 prefix sum with DPP (VALU-rate lane moves, no LDS):
// Hillis-Steele inside each 16-lane row (row_shr 1,2,4,8), then
// row_bcast:15 / row_bcast:31 carry row totals across rows (gfx9 family).
template <int Ctrl, int RowMask, int BankMask>
__device__ __forceinline__ uint32_t dpp_add(uint32_t v) {
  return v + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, Ctrl, RowMask, BankMask, false);
}
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  v = dpp_add<0x111, 0xf, 0xf>(v);   // row_shr:1
  v = dpp_add<0x112, 0xf, 0xf>(v);   // row_shr:2
  v = dpp_add<0x114, 0xf, 0xf>(v);   // row_shr:4
  v = dpp_add<0x118, 0xf, 0xf>(v);   // row_shr:8
  v = dpp_add<0x142, 0xa, 0xf>(v);   // row_bcast:15 -> rows 1, 3
  v = dpp_add<0x143, 0xc, 0xf>(v);   // row_bcast:31 -> rows 2, 3
  return v;
}

// exclusive scan over an NB-thread block; `wsum` is LDS[NB / 64].  kTrail =
// false skips the closing barrier: for a `wsum` whose next scan is already
// ordered after this one's reads by some other barrier.
template <bool kTrail = true, int NB = kBlock>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* wsum, uint32_t& total) {
  const uint32_t inc = wave_incl_scan(v);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t off = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < NB / 64; ++k) {
    const uint32_t x = wsum[k];
    off += (k < w) ? x : 0u;
    tot += x;
  }
  if (kTrail) __syncthreads();
  total = tot;
  return off + inc - v;
}

// Per-frame camera constants for unprojection (spec, same in csg_oracle.c):
// camera-to-world rotation = transpose of the view rotation, camera position
// c_i = -((V0i*t0 + V1i*t1) + V2i*t2), and fx, fy, cx, cy read back from the
// pixel projection (rows u*w = fx*x - cx*z, v*w = -fy*y - cy*z, w = -z).
__device__ __forceinline__ void frame_camera(const float* V, const float* P, float* cam) {
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int j = 0; j < 3; ++j) cam[i * 3 + j] = V[j * 4 + i];
    cam[9 + i] = -((V[0 * 4 + i] * V[3] + V[1 * 4 + i] * V[7]) + V[2 * 4 + i] * V[11]);
  }
  cam[12] = P[0];
  cam[13] = -P[5];
  cam[14] = -P[2];
  cam[15] = -P[6];
}

// World-space point on the ray through pixel (px, py)'s centre at distance-to-
// image-plane d.
__device__ __forceinline__ void unproject(const float* cam, int px, int py, float d, float out[3]) {
  const float a = ((float)px + 0.5f) - cam[14], bq = ((float)py + 0.5f) - cam[15];
  const float xc = (a * d) / cam[12], yc = -((bq * d) / cam[13]), zc = -d;
#pragma unroll
  for (int i = 0; i < 3; ++i) out[i] = ((cam[i * 3 + 0] * xc + cam[i * 3 + 1] * yc) + cam[i * 3 + 2] * zc) + cam[9 + i];
}

// f16 bits of x rounded to nearest even; -0 is canonicalised to +0 first
// (the spec's outputs carry no negative zeros).
__device__ __forceinline__ uint32_t half_bits(float x) {
  const _Float16 h = (_Float16)(x + 0.0f);   // v_cvt_f16_f32, round to nearest even
  return (uint32_t)__builtin_bit_cast(uint16_t, h);
}

// ---------------------------------------------------------------------------
// k_clip: per (frame, instance) clip rows of P*V*M; per frame P*V
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_clip(SceneDev s, BatchDev b) {
  const uint32_t f = blockIdx.y;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const FrameDev& fr = b.frames[f];
  // A device-side frame record can name any set: out-of-range sets render with
  // set 0 and raise kOvBadSet (csg_synchronize reports it); every later kernel
  // reads the checked set from b.fset.
  const uint32_t raw = fr.xform_set;
  const uint32_t set = raw < b.n_sets ? raw : 0u;
  if (i < s.n_inst) {
    const float* M = b.models + ((size_t)set * s.n_inst + i) * 16;
    float m[16], vm[16], c[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) m[k] = M[k];
    mat4_mul(fr.view, m, vm);
    mat4_mul(fr.proj, vm, c);
    float* o = b.clip + ((size_t)f * s.n_inst + i) * 12;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      o[k] = c[k];
      o[4 + k] = c[4 + k];
      o[8 + k] = c[12 + k];
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    b.fset[f] = set;
    if (raw >= b.n_sets) atomicOr(b.overflow, kOvBadSet);
    float pv[16];
    mat4_mul(fr.proj, fr.view, pv);
    float* o = b.pv + (size_t)f * 12;
    for (int k = 0; k < 4; ++k) {
      o[k] = pv[k];
      o[4 + k] = pv[4 + k];
      o[8 + k] = pv[12 + k];
    }
    frame_camera(fr.view, fr.proj, b.cam + (size_t)f * kCamFloats);
  }
}

// ---------------------------------------------------------------------------
// k_setup
// ---------------------------------------------------------------------------
// Build one raster record from screen-space vertices; false if it covers no pixel.
// Groups 0-1 of a raster record (x0 x1 x2 y0 | y1 y2 p0 p1): the part that
// differs between the sub-triangles of one clipped triangle.
struct SubRec { uint4 g0, g1; };

__device__ __forceinline__ bool make_rec(const SceneDev& s, const float* su, const float* sv, SubRec& r) {
  int32_t x[3], y[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    if (!(fabsf(su[k]) < kGuardPx) || !(fabsf(sv[k]) < kGuardPx)) return false;
    x[k] = (int32_t)rintf(su[k] * 256.0f);
    y[k] = (int32_t)rintf(sv[k] * 256.0f);
  }
  const int64_t area = (int64_t)(x[1] - x[0]) * (y[2] - y[0]) - (int64_t)(x[2] - x[0]) * (y[1] - y[0]);
  if (area == 0) return false;
  if (area < 0) {
    int32_t t = x[1]; x[1] = x[2]; x[2] = t;
    t = y[1]; y[1] = y[2]; y[2] = t;
  }
  const int32_t xmin = min(x[0], min(x[1], x[2])), xmax = max(x[0], max(x[1], x[2]));
  const int32_t ymin = min(y[0], min(y[1], y[2])), ymax = max(y[0], max(y[1], y[2]));
  int px0 = (xmin - 128 + 255) >> 8, px1 = (xmax - 128) >> 8;
  int py0 = (ymin - 128 + 255) >> 8, py1 = (ymax - 128) >> 8;
  px0 = max(px0, 0);
  py0 = max(py0, 0);
  px1 = min(px1, (int)s.W - 1);
  py1 = min(py1, (int)s.H - 1);
  if (px0 > px1 || py0 > py1) return false;
  // Small records (at most NxN pixel centres in the box, vertex extent below
  // 32 px): evaluate the spec's edge test at every centre of the box, drop the
  // record if it covers none and shrink the box to the covered pixels.  The
  // covered set is unchanged (so are the outputs); fewer, tighter records mean
  // fewer record stores, bin entries and raster row items.  Exact in int32:
  // |dx|, |dy| < 2^13 and every centre lies within the vertex extent.
  constexpr int N = kSmallCover;
  if (px1 - px0 < N && py1 - py0 < N && xmax - xmin < 8192 && ymax - ymin < 8192) {
    const int32_t cx0 = px0 * 256 + 128, cy0 = py0 * 256 + 128;
    const int ea[3] = {1, 2, 0}, eb[3] = {2, 0, 1};
    int32_t e0[3], sx[3], sy[3];
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      const int32_t dx = x[eb[e]] - x[ea[e]], dy = y[eb[e]] - y[ea[e]];
      const int32_t bias = (dy < 0 || (dy == 0 && dx > 0)) ? 0 : -1;
      e0[e] = __mul24(dx, cy0 - y[ea[e]]) - __mul24(dy, cx0 - x[ea[e]]) + bias;
      sx[e] = -dy * 256;
      sy[e] = dx * 256;
    }
    const int nw = px1 - px0, nh = py1 - py0;
    uint32_t cols = 0, rows = 0;
    // the active lanes' largest box, wave-uniform: a wave of 1x1 and 2x2 boxes
    // evaluates 1 or 4 centres, not N*N
    int nwm = 0, nhm = 0;
#pragma unroll
    for (int k = 1; k < N; ++k) {
      nwm += __any(nw >= k) ? 1 : 0;
      nhm += __any(nh >= k) ? 1 : 0;
    }
    // E(i, j) = e0 + sx*i + sy*j stepped by additions (the same integers; a
    // constant multiple such as sx*3 otherwise became a quarter-rate v_mul_lo_u32)
    int32_t er[3] = {e0[0], e0[1], e0[2]};
#pragma unroll
    for (int j = 0; j < N; ++j) {
      if (j > nhm) break;
      int32_t ec[3] = {er[0], er[1], er[2]};
#pragma unroll
      for (int i = 0; i < N; ++i) {
        if (i > nwm) break;
        const bool in = i <= nw && j <= nh && (ec[0] | ec[1] | ec[2]) >= 0;
        cols |= in ? 1u << i : 0u;
        rows |= in ? 1u << j : 0u;
#pragma unroll
        for (int e = 0; e < 3; ++e) ec[e] += sx[e];
      }
#pragma unroll
      for (int e = 0; e < 3; ++e) er[e] += sy[e];
    }
    if (!cols) return false;
    px1 = px0 + 31 - __clz(cols);
    px0 += __ffs(cols) - 1;
    py1 = py0 + 31 - __clz(rows);
    py0 += __ffs(rows) - 1;
  }
  r.g0 = make_uint4((uint32_t)x[0], (uint32_t)x[1], (uint32_t)x[2], (uint32_t)y[0]);
  r.g1 = make_uint4((uint32_t)y[1], (uint32_t)y[2], (uint32_t)px0 | ((uint32_t)py0 << 16),
                    (uint32_t)px1 | ((uint32_t)py1 << 16));
  return true;
}

// Tile rectangle of a record: tx0 | ty0 << 8 | tx1 << 16 | ty1 << 24, 8-bit
// tile coordinates.  Frames of more than 256 tile rows (taller than 4,096 px
// at 32 x 16; at most 512 rows) store tile-row PAIRS (ys = 1, SceneDev::
// rect_ys): the record is binned to both tiles of every pair its box touches,
// a superset the raster's per-tile row clipping makes harmless (a record
// binned to a tile it misses stages no rows), so outputs do not change.
__device__ __forceinline__ uint32_t rec_tile_rect(const SubRec& r, uint32_t ys) {
  const uint32_t px0 = r.g1.z & 0xFFFFu, py0 = r.g1.z >> 16, px1 = r.g1.w & 0xFFFFu, py1 = r.g1.w >> 16;
  return (px0 / kTileW) | (((py0 / kTileH) >> ys) << 8) | ((px1 / kTileW) << 16) | (((py1 / kTileH) >> ys) << 24);
}

// first and last tile row of a rectangle (rows past the frame's last dropped)
__device__ __forceinline__ uint32_t rect_ty0(uint32_t rc, uint32_t ys) { return ((rc >> 8) & 255u) << ys; }
__device__ __forceinline__ uint32_t rect_ty1(uint32_t rc, uint32_t ys, uint32_t tiles_y) {
  return min((((rc >> 24) + 1u) << ys) - 1u, tiles_y - 1u);
}

__device__ __forceinline__ uint32_t rect_area(uint32_t rc, uint32_t ys, uint32_t tiles_y) {
  const uint32_t tx0 = rc & 255u, tx1 = (rc >> 16) & 255u;
  return (tx1 - tx0 + 1) * (rect_ty1(rc, ys, tiles_y) - rect_ty0(rc, ys) + 1);
}

// q / w for q < 2^24, 1 <= w <= 256: float reciprocal estimate (off by at
// most one), then one exact correction (no integer division sequence)
__device__ __forceinline__ uint32_t small_div(uint32_t q, uint32_t w) {
  uint32_t d = (uint32_t)((float)q * __builtin_amdgcn_rcpf((float)w));
  const uint32_t p = __umul24(d, w);
  d = p > q ? d - 1u : (p + w <= q ? d + 1u : d);
  return d;
}

__device__ __forceinline__ uint32_t rect_tile(uint32_t rc, uint32_t q, uint32_t tiles_x, uint32_t ys) {
  const uint32_t tx0 = rc & 255u, ty0 = rect_ty0(rc, ys), tx1 = (rc >> 16) & 255u;
  const uint32_t w = tx1 - tx0 + 1;
  const uint32_t r = small_div(q, w);
  return __umul24(ty0 + r, tiles_x) + tx0 + (q - __umul24(r, w));
}

typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
// Chunk cull of one (frame, chunk): true if all 8 corners of the chunk's
// object-space AABB fail one frustum plane by a margin -- then every triangle
// inside would fail that plane in the per-triangle test too, so the output is
// unchanged.  Corner c of the box (x from bit 2, y bit 1, z bit 0).  (Measured:
// per-64-triangle slice AABBs cull more but cost more than they save.)
struct CullOut { bool n, f, l, r, t, b; };
__device__ __forceinline__ CullOut corner_out(const SceneDev& s, const Chunk& ch, const float* Cm, int c) {
  const float px = (c & 4) ? ch.hi[0] : ch.lo[0];
  const float py = (c & 2) ? ch.hi[1] : ch.lo[1];
  const float pz = (c & 1) ? ch.hi[2] : ch.lo[2];
  const float X = dot4(Cm + 0, px, py, pz), Y = dot4(Cm + 4, px, py, pz), Wc = dot4(Cm + 8, px, py, pz);
  const float tol = 1e-3f * (fabsf(X) + fabsf(Y) + fabsf(Wc)) + 1e-3f;
  return CullOut{Wc < s.near_clip - tol, Wc > s.far_clip + tol, X < -tol, X > (float)s.W * Wc + tol * (float)s.W,
                 Y < -tol, Y > (float)s.H * Wc + tol * (float)s.H};
}

// The spec's per-vertex 1/W (spec 3): W >= near_clip > 2^-126 after near-plane
// clipping, so below 2^126 the Newton reciprocal is the IEEE one (rcp_ieee);
// the division only past that (never taken by real scenes: a uniform branch)
__device__ __forceinline__ float rcp_w(float w) { return w <= 0x1p126f ? rcp_ieee(w) : 1.0f / w; }

// The records of one chunk of triangles for frame f (one triangle per thread
// of a 256-thread block; `sw` is the calling wave's record stage).  (A
// per-vertex variant -- each slice's distinct vertices transformed once into
// LDS -- was bit-exact and 8% slower: profiles/r06/ab/setup_verts.txt.)
__device__ __forceinline__ void setup_chunk(const SceneDev& s, const BatchDev& b, const Chunk& ch, uint32_t f,
                                            int tid, int lane, uint4* sw);

// Grid: x = frame (fast), (y, z) = chunk.  Consecutive workgroups take the
// same chunk for successive frames, so a chunk's triangles (and its clip
// rows' instance) are read from HBM once and then hit in L2 (measured on C3:
// 0.45 vs 0.73 ms per 60 frames with the chunk index fast).
__global__ __launch_bounds__(256) void k_setup(SceneDev s, BatchDev b, const Chunk* __restrict__ chunks,
                                               uint32_t n_chunks) {
  const uint32_t f = blockIdx.x, chunk = blockIdx.y + blockIdx.z * gridDim.y;
  if (chunk >= n_chunks) return;
  const int tid = threadIdx.x, lane = tid & 63;
  if (DBG(b.dbg) & 32u) return;            // ablation: empty setup
  const Chunk& ch = chunks[chunk];   // read fields in place (a runtime-indexed copy would spill)
  // every wave evaluates the 8 corners (lanes 0-7); the block leaves together
  {
    const CullOut o = corner_out(s, ch, b.clip + ((size_t)f * s.n_inst + ch.inst) * 12, lane & 7);
    const uint64_t m8 = 0xFFull;
    const bool cull = ((__ballot(o.n) & m8) == m8) || ((__ballot(o.f) & m8) == m8) ||
                      ((__ballot(o.l) & m8) == m8) || ((__ballot(o.r) & m8) == m8) ||
                      ((__ballot(o.t) & m8) == m8) || ((__ballot(o.b) & m8) == m8);
    if (cull || (DBG(b.dbg) & 64u)) return;   // identical in every wave of the block (64: ablation, cull all)
  }
  static_assert(16 * kRecGroups <= 2 * 64, "two chunk stores per lane");
  __shared__ uint4 tstage[kBlock / 64][16 * kRecGroups];
  setup_chunk(s, b, ch, f, tid, lane, tstage[tid >> 6]);
}

__device__ __forceinline__ void setup_chunk(const SceneDev& s, const BatchDev& b, const Chunk& ch, uint32_t f,
                                            int tid, int lane, uint4* sw) {
  const uint32_t i = ch.inst;
  const float* Cm = b.clip + ((size_t)f * s.n_inst + i) * 12;

  // Records: groups 0-1 per sub-triangle (r0, r1: named, never runtime-
  // indexed, which would put them in scratch), groups 2-4 shared (the
  // original triangle's uid, alpha texture and planes).
  SubRec r0, r1;
  uint4 c2 = make_uint4(0u, 0u, 0u, 0u), c3 = c2, c4 = c2;
  int nrec = 0;
  if ((uint32_t)tid < ch.count) {
    const uint32_t g = ch.soup + tid;   // soup index (no instance-table load on the way)
    Cv3 v[3];
    float c[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) c[k] = Cm[k];
    const float* tp = s.tri_pos + (size_t)g * 9;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float px = tp[3 * k], py = tp[3 * k + 1], pz = tp[3 * k + 2];
      v[k].x = dot4(c + 0, px, py, pz);
      v[k].y = dot4(c + 4, px, py, pz);
      v[k].w = dot4(c + 8, px, py, pz);
    }
    const float nearc = s.near_clip, farc = s.far_clip;
    const float Wf = (float)s.W, Hf = (float)s.H;
    bool on = true, of = true, ol = true, orr = true, ot = true, ob = true;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      on &= v[k].w < nearc;
      of &= v[k].w > farc;
      ol &= v[k].x < 0.0f;
      orr &= v[k].x > Wf * v[k].w;
      ot &= v[k].y < 0.0f;
      ob &= v[k].y > Hf * v[k].w;
    }
    if ((DBG(b.dbg) & 0x10000u) && !(on | of | ol | orr | ot | ob)) {   // ablation: stop after the frustum test
      if (v[0].x == 1.2345e-30f && b.inst) b.inst[0] = 1;              // (keeps the transform live)
    } else if (!(on | of | ol | orr | ot | ob)) {
      const uint32_t uid = (i << s.uid_shift) | g;
      // Sutherland-Hodgman against W >= near over edges v0->v1, v1->v2, v2->v0
      // (each edge emits [start vertex if inside][intersection if crossing]),
      // written as a closed-form case table on the inside mask so the polygon
      // stays in registers.
      Cv3 q0 = v[0], q1 = v[1], q2 = v[2], q3 = v[2];
      int nq = 3;
      const bool in0 = v[0].w >= nearc, in1 = v[1].w >= nearc, in2 = v[2].w >= nearc;
      if (!(in0 && in1 && in2)) {
        auto cross_pt = [&](const Cv3& a, const Cv3& bb) {
          const float tt = (nearc - a.w) / (bb.w - a.w);
          Cv3 rr;
          rr.x = a.x + tt * (bb.x - a.x);
          rr.y = a.y + tt * (bb.y - a.y);
          rr.w = nearc;
          return rr;
        };
        auto sel = [](bool c, const Cv3& a, const Cv3& bb) {
          Cv3 rr;
          rr.x = c ? a.x : bb.x;
          rr.y = c ? a.y : bb.y;
          rr.w = c ? a.w : bb.w;
          return rr;
        };
        const Cv3 I01 = cross_pt(v[0], v[1]), I12 = cross_pt(v[1], v[2]), I20 = cross_pt(v[2], v[0]);
        const int code = (int)in0 | ((int)in1 << 1) | ((int)in2 << 2);
        // code: 1 -> v0 I01 I20 | 2 -> I01 v1 I12 | 4 -> I12 v2 I20
        //       3 -> v0 v1 I12 I20 | 6 -> I01 v1 v2 I20 | 5 -> v0 I01 I12 v2
        q0 = sel(code == 2 || code == 6, I01, sel(code == 4, I12, v[0]));
        q1 = sel(code == 1 || code == 5, I01, sel(code == 4, v[2], v[1]));
        q2 = sel(code == 1 || code == 4, I20, sel(code == 6, v[2], I12));
        q3 = sel(code == 3 || code == 6, I20, v[2]);
        nq = (code == 1 || code == 2 || code == 4) ? 3 : 4;
      }
      // spec 3: one IEEE reciprocal per vertex, u = X * (1/W) (as csg_oracle.c)
      auto emit_tri_r = [&](const Cv3& a, float ra, const Cv3& bb, float rb, const Cv3& cc, float rc) {
        float su[3], sv[3];
        su[0] = a.x * ra; sv[0] = a.y * ra;
        su[1] = bb.x * rb; sv[1] = bb.y * rb;
        su[2] = cc.x * rc; sv[2] = cc.y * rc;
        SubRec rr;
        if (make_rec(s, su, sv, rr)) {
          if (nrec == 0) r0 = rr; else r1 = rr;
          ++nrec;
        }
      };
      auto emit_tri = [&](const Cv3& a, const Cv3& bb, const Cv3& cc) {
        emit_tri_r(a, rcp_w(a.w), bb, rcp_w(bb.w), cc, rcp_w(cc.w));
      };
      if (nq >= 3) emit_tri(q0, q1, q2);
      if (nq >= 4) emit_tri(q0, q2, q3);
      // A record exists iff det != 0 and the screen test passes, in either
      // order: the homogeneous setup, its IEEE reciprocal and the material
      // loads are spent only on the few triangles that cover a pixel centre
      // (about one in five of those that pass the frustum test).
      if (nrec > 0) {
        Hom h;
        hom_setup(v, h);
        if (!h.ok) {
          nrec = 0;
        } else {
          const InstSetDev is = b.iset[(size_t)b.fset[f] * s.n_inst + i];
          // a threshold of 255 passes no fragment: such a record is not emitted
          const uint32_t atex = is.atex == kNoAlpha ? kNoAlpha : rec_atex(is.atex, is.athr), atex_wh = is.atex_wh;
          if (is.atex != kNoAlpha && is.athr >= 255u) nrec = 0;
          float D[3], U[3] = {0.0f, 0.0f, 0.0f}, V[3] = {0.0f, 0.0f, 0.0f};
          depth_plane(h.A, h.B, h.C, h.invdet, D);
          if (is.alpha_uv) {   // uvs loaded only now: few values live at once
            const float* tu = s.tri_uv + (size_t)g * 6;
            float uv[6];
#pragma unroll
            for (int k = 0; k < 6; ++k) uv[k] = tu[k];
            uv_planes(h.A, h.B, h.C, h.invdet, uv, U, V);
          }
          c2 = make_uint4(uid, atex, __float_as_uint(D[0]), __float_as_uint(D[1]));
          c3 = make_uint4(__float_as_uint(U[0]), __float_as_uint(V[0]), __float_as_uint(U[1]), __float_as_uint(V[1]));
          c4 = make_uint4(__float_as_uint(U[2]), __float_as_uint(V[2]), __float_as_uint(D[2]), atex_wh);
        }
      }
    }
  }
  // wave-ballot compaction of the emitted records into the frame's record list
  const uint64_t b1 = __ballot(nrec >= 1), b2 = __ballot(nrec >= 2);
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const uint32_t mine = (uint32_t)(__popcll(b1 & lt) + __popcll(b2 & lt));
  const uint32_t wtot = (uint32_t)(__popcll(b1) + __popcll(b2));
  uint32_t wbase = 0;
  if (lane == 0 && wtot) wbase = atomicAdd(&b.rec_count[f * kCounterStride], wtot);
  wbase = __shfl(wbase, 0, 64);
  if (DBG(b.dbg) & 128u) {   // ablation: no record stores
    if (nrec == 3 && b.inst) b.inst[0] = r0.g0.x + r1.g0.x + c2.x + c3.x + c4.x;
    return;
  }
  // Coalesced record stores.  The wave's records take the contiguous slots
  // [wbase, wbase + wtot), but lane-by-lane 16-B stores at an 80-B stride
  // write many more partial 128-B lines than the bytes need.  So, 16 records
  // at a time, the lanes holding them put them in a per-wave LDS stage and the
  // wave stores the stage as consecutive 16-B chunks (1 KB per instruction),
  // non-temporally: whole lines that would otherwise push the chunk's
  // triangles, which the next frames' workgroups re-read, out of L2 (setup
  // -1.1%, profiles/r03/ab/nt_record_stores.txt; round 1's non-temporal stores
  // of scattered 112-B records were 5x slower: partial lines).
  // Wave-local: the loop count is uniform per wave, so there is no block barrier.
  const uint64_t rbase = b.slab[f].rec_base;
  const uint32_t rcap = b.slab[f].rec_cap;
  if (lane == 0 && wbase + wtot > rcap) atomicOr(b.overflow, 1u);
  uint4* dst = reinterpret_cast<uint4*>(b.recs + rbase);
  const size_t lim = (size_t)rcap * kRecGroups;
  auto put = [&](uint32_t at, const SubRec& r) {
    uint4* o = sw + at * kRecGroups;
    o[0] = r.g0;
    o[1] = r.g1;
    o[2] = c2;
    o[3] = c3;
    o[4] = c4;
  };
  for (uint32_t p0 = 0; p0 < wtot; p0 += 16) {
    if (nrec > 0 && mine - p0 < 16u) put(mine - p0, r0);
    if (nrec > 1 && mine + 1u - p0 < 16u) put(mine + 1u - p0, r1);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const uint32_t nch = min(16u, wtot - p0) * kRecGroups;
    const size_t at = ((size_t)wbase + p0) * kRecGroups;
#pragma unroll
    for (uint32_t c = (uint32_t)lane; c < 2u * 64u; c += 64u)
      if (c < nch && at + c < lim) {   // non-temporal: k_raster reads them long after L2 has turned over
        const uint4 q = sw[c];
        const v4u32 w = {q.x, q.y, q.z, q.w};
        __builtin_nontemporal_store(w, reinterpret_cast<v4u32*>(dst + at + c));
      }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  if (nrec > 0 && wbase + mine < rcap) b.rect[rbase + wbase + mine] = rec_tile_rect(r0, s.rect_ys);
  if (nrec > 1 && wbase + mine + 1 < rcap) b.rect[rbase + wbase + mine + 1] = rec_tile_rect(r1, s.rect_ys);
}

// ---------------------------------------------------------------------------
// Binning rounds.  A round takes kBinRpt = 4 records per thread (kBinRound per
// block, each thread's records consecutive: one 16-B load of their tile
// rects), scans their tile counts into pre[] and expands (record, tile) items
// with a 4-ary search.  Bigger rounds mean fewer barriers and tile sweeps per
// block (measured: 1 record per thread, bin +6%).
// ---------------------------------------------------------------------------
constexpr int kBinRpt = 4;
constexpr uint32_t kBinRound = kBlock * kBinRpt;
// k_count / k_bin keep one LDS counter per tile.  A workgroup may hold at most
// 160 KiB of LDS, so frames of more than kBinBand tiles (16.8 M pixels at
// 32x16, e.g. 8192 x 2048; the limit is 256 x 256 tiles) are binned in bands
// of kBinBand tiles:
// each band re-reads the 4-B tile rectangles and counts / places only the
// entries of its own tiles.  Below that (every BASELINE workload) there is one
// band and the kernels run as before.
constexpr uint32_t kBinBand = 32768;

// last k in [0, kBinRound) with pre[k] <= j (pre: kBinRound + 1 entries,
// nondecreasing).  4-ary search: each step issues three independent LDS reads,
// so the dependent chain is 5 LDS round trips instead of 10.
__device__ __forceinline__ int find_bin_item(const uint32_t* pre, uint32_t j) {
  int lo = 0;
#pragma unroll
  for (int step = 256; step > 0; step >>= 2) {
    const uint32_t a = pre[lo + step], b2 = pre[lo + 2 * step], c = pre[lo + 3 * step];
    lo += ((a <= j) + (b2 <= j) + (c <= j)) * step;
  }
  return lo;
}

// Load this thread's records of the round at `base` (record ids base + tid*kBinRpt + q),
// fill lrc[] and pre[]; returns the round's item total.  With kSingle, a
// record touching at most kCountDirect tiles (most of them) is not expanded:
// its own thread calls `single(q, tile)` for each tile.  k_count does so (its
// counts do not depend on the order; C3: binning 0.64 -> 0.52 ms, frames/s
// +0.8%); k_bin expands every record, so a tile's list keeps the record order
// the raster is tuned for (binning single-tile records directly in k_bin too,
// in or out of record order, saved at most 0.07 ms there and cost as much raster).
constexpr uint32_t kCountDirect = 4;
template <uint32_t kDirect, typename Single>
__device__ __forceinline__ uint32_t bin_round_setup(const uint32_t* rect, uint32_t base, uint32_t n, uint32_t* lrc,
                                                    uint32_t* pre, uint32_t* wsum, const SceneDev& s, Single single) {
  const int tid = threadIdx.x;
  const uint32_t r0 = base + (uint32_t)tid * kBinRpt;
  uint32_t rc[kBinRpt], area[kBinRpt], sum = 0;
  static_assert(kBinRpt == 4, "one 16-B rect load per thread");
  uint4 v = make_uint4(0u, 0u, 0u, 0u);
  if (r0 + 3 < n) {
    v = *reinterpret_cast<const uint4*>(rect + r0);   // rect rows are 16-B aligned (slab bases % 4 == 0)
  } else {
    if (r0 < n) v.x = rect[r0];
    if (r0 + 1 < n) v.y = rect[r0 + 1];
    if (r0 + 2 < n) v.z = rect[r0 + 2];
  }
  rc[0] = v.x; rc[1] = v.y; rc[2] = v.z; rc[3] = v.w;
#pragma unroll
  for (int q = 0; q < kBinRpt; ++q) {
    area[q] = (r0 + (uint32_t)q < n) ? rect_area(rc[q], s.rect_ys, s.tiles_y) : 0u;
    lrc[tid * kBinRpt + q] = rc[q];
    if (kDirect && area[q] && area[q] <= kDirect) {
#pragma clang loop unroll(disable)
      for (uint32_t a = 0; a < area[q]; ++a) single(q, rect_tile(rc[q], a, s.tiles_x, s.rect_ys));
      area[q] = 0u;
    }
  }
#pragma unroll
  for (int q = 0; q < kBinRpt; ++q) sum += area[q];
  uint32_t total;
  uint32_t ex = block_excl_scan(sum, wsum, total);
#pragma unroll
  for (int q = 0; q < kBinRpt; ++q) {
    pre[tid * kBinRpt + q] = ex;
    ex += area[q];
  }
  if (tid == kBlock - 1) pre[kBinRound] = ex;
  return total;
}

// ---------------------------------------------------------------------------
// k_count: per-tile record counts (LDS-aggregated, grid-stride over a frame's records)
// ---------------------------------------------------------------------------
template <bool kBanded>
__global__ __launch_bounds__(256) void k_count(SceneDev s, BatchDev b) {
  extern __shared__ __attribute__((aligned(16))) uint32_t dyn_count[];
  const uint32_t band = min(s.n_tiles, kBinBand);
  uint32_t* hist = dyn_count;                          // [band]
  uint32_t* pre = dyn_count + ((band + 3u) & ~3u);     // [kBinRound + 1]
  uint32_t* lrc = pre + kBinRound + 4;                 // [kBinRound]
  uint32_t* wsum = lrc + kBinRound;                    // [4]
  const uint32_t f = blockIdx.y;
  const int tid = threadIdx.x;
  const uint32_t n = min(b.rec_count[f * kCounterStride], b.slab[f].rec_cap);
  const uint32_t* rect = b.rect + b.slab[f].rec_base;
  // this block's row of the count grid (k_colscan turns it into offsets)
  uint32_t* bc = b.bcount + ((size_t)f * gridDim.x + blockIdx.x) * s.n_tiles;
  for (uint32_t t0 = 0; t0 < s.n_tiles; t0 += band) {
    const uint32_t nb = min(band, s.n_tiles - t0);   // tiles [t0, t0 + nb)
    for (uint32_t t = tid; t < nb; t += kBlock) hist[t] = 0;
    __syncthreads();
    for (uint32_t base = blockIdx.x * kBinRound; base < n; base += gridDim.x * kBinRound) {
      const uint32_t total = bin_round_setup<kCountDirect>(rect, base, n, lrc, pre, wsum, s,
                                                   [&](int, uint32_t t) {
                                                     if (!kBanded || t - t0 < nb) atomicAdd(&hist[t - t0], 1u);
                                                   });
      __syncthreads();
      for (uint32_t j = tid; j < total; j += kBlock) {
        const int k = find_bin_item(pre, j);
        const uint32_t t = rect_tile(lrc[k], j - pre[k], s.tiles_x, s.rect_ys);
        if (!kBanded || t - t0 < nb) atomicAdd(&hist[t - t0], 1u);
      }
      __syncthreads();
    }
    for (uint32_t t = tid; t < nb; t += kBlock) bc[t0 + t] = hist[t];
    __syncthreads();   // (the next band zeroes hist)
  }
}

// Column scan of the count grid: per tile, the exclusive prefix over the
// k_count blocks (in block order, so each block's entries of a tile take a
// fixed range of its list) and the tile's total.  Grid (tile groups, F).
__global__ __launch_bounds__(256) void k_colscan(SceneDev s, BatchDev b) {
  const uint32_t f = blockIdx.y, t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= s.n_tiles) return;
  uint32_t* col = b.bcount + (size_t)f * b.bin_blocks * s.n_tiles + t;
  uint32_t run = 0;
#pragma unroll 8
  for (uint32_t k = 0; k < b.bin_blocks; ++k) {
    const uint32_t v = col[(size_t)k * s.n_tiles];
    col[(size_t)k * s.n_tiles] = run;
    run += v;
  }
  b.tile_count[(size_t)f * s.n_tiles + t] = run;
}

// ---------------------------------------------------------------------------
// k_plan: each frame's slab of the chain's record and bin pools, packed back
// to back in frame order.  A frame's caps are its hints (csg_size_work wrote
// them into the frame record: the measured counts with the margin) or the
// context's per-frame caps.  One wave: 64 frames per step, a 64-bit
// inclusive scan over the wave, a running base.  A frame past a pool's end
// gets what is left (possibly nothing): k_setup / k_scan flag its overflow.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t wave_incl_scan64(uint64_t v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

__global__ __launch_bounds__(64) void k_plan(const FrameDev* __restrict__ frames, uint32_t F, uint32_t def_rec,
                                             uint32_t def_bin, uint64_t rec_pool, uint64_t bin_pool, int use_hints,
                                             Slab* __restrict__ slab, uint64_t* __restrict__ need) {
  const int lane = threadIdx.x;
  uint64_t cr = 0, cb = 0;
  for (uint32_t f0 = 0; f0 < F; f0 += 64) {
    const uint32_t f = f0 + (uint32_t)lane;
    uint32_t rc = 0, bc = 0;
    if (f < F) {
      const uint32_t rh = use_hints ? frames[f].records_hint : 0u, bh = use_hints ? frames[f].bins_hint : 0u;
      rc = rh ? ((min(rh, 0x7FFFFFF0u) + 3u) & ~3u) : def_rec;
      bc = bh ? ((min(bh, 0x7FFFFFF0u) + 3u) & ~3u) : def_bin;
    }
    const uint64_t ir = wave_incl_scan64(rc, lane), ib = wave_incl_scan64(bc, lane);
    if (f < F) {
      Slab sl;
      sl.rec_base = min(cr + ir - rc, rec_pool);
      sl.bin_base = min(cb + ib - bc, bin_pool);
      sl.rec_cap = (uint32_t)min((uint64_t)rc, rec_pool - sl.rec_base);
      sl.bin_cap = (uint32_t)min((uint64_t)bc, bin_pool - sl.bin_base);
      sl.pad[0] = sl.pad[1] = 0u;
      slab[f] = sl;
    }
    cr += __shfl(ir, 63, 64);
    cb += __shfl(ib, 63, 64);
  }
  // the largest chain of the batch (chains run one after another on the
  // stream; the host zeroes need[] before a batch and reads it on overflow)
  if (lane == 0) {
    need[0] = max(need[0], cr);
    need[1] = max(need[1], cb);
  }
}

// ---------------------------------------------------------------------------
// k_scan: per frame exclusive scan of tile counts (one 256-thread block)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_scan(SceneDev s, BatchDev b) {
  __shared__ uint32_t wsum[kBlock / 64];
  __shared__ uint32_t carry;
  const uint32_t f = blockIdx.x;
  const uint32_t* tc = b.tile_count + (size_t)f * s.n_tiles;
  uint32_t* to = b.tile_off + (size_t)f * (s.n_tiles + 1);
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint32_t base = 0; base < s.n_tiles; base += kBlock) {
    const uint32_t t = base + threadIdx.x;
    const uint32_t v = t < s.n_tiles ? tc[t] : 0u;
    uint32_t tot;
    const uint32_t ex = block_excl_scan(v, wsum, tot);
    const uint32_t c0 = carry;
    if (t < s.n_tiles) to[t] = c0 + ex;
    __syncthreads();
    if (threadIdx.x == 0) carry = c0 + tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    to[s.n_tiles] = carry;
    if (carry > b.slab[f].bin_cap) atomicOr(b.overflow, 2u);
  }
}

// ---------------------------------------------------------------------------
// k_bin: scatter record ids into per-tile bins.  Each tile's next free slot
// for this block comes from the count grid (the tile's list start plus the
// entries of the blocks before it, k_colscan): LDS atomics only, no global
// atomics, and each block's entries of a tile are a fixed range of its list.
// ---------------------------------------------------------------------------
template <bool kBanded>
__global__ __launch_bounds__(256) void k_bin(SceneDev s, BatchDev b) {
  extern __shared__ uint32_t dyn[];
  uint32_t* hist = dyn;                  // [band] next slot of each tile of the band
  __shared__ uint32_t pre[kBinRound + 1];
  __shared__ uint32_t lrc[kBinRound];
  __shared__ uint32_t wsum[kBlock / 64];
  const uint32_t f = blockIdx.y;
  const int tid = threadIdx.x;
  const Slab sb = b.slab[f];
  const uint32_t n = min(b.rec_count[f * kCounterStride], sb.rec_cap);
  const uint32_t* rect = b.rect + sb.rec_base;
  const uint32_t* toff = b.tile_off + (size_t)f * (s.n_tiles + 1);
  uint32_t* bins = b.bins + sb.bin_base;
  const uint32_t* bo = b.bcount + ((size_t)f * gridDim.x + blockIdx.x) * s.n_tiles;
  // Reverse append order: this block's range mirrored, filled from its end.
  // Outputs do not depend on the order (the z-buffer minimum and the coverage
  // bits are order-independent); the raster is measurably faster this way
  // (-0.8% on C3: the scene's small foreground proxies, appended last, reach
  // the z-buffer first).
  const uint32_t* tcnt = b.tile_count + (size_t)f * s.n_tiles;
  const uint32_t band = min(s.n_tiles, kBinBand);
  for (uint32_t t0 = 0; t0 < s.n_tiles; t0 += band) {
    const uint32_t nb = min(band, s.n_tiles - t0);   // tiles [t0, t0 + nb)
    for (uint32_t t = tid; t < nb; t += kBlock)
      hist[t] = toff[t0 + t] + tcnt[t0 + t] - bo[t0 + t] - 1u;   // last slot of the mirrored range; decremented
    __syncthreads();
    for (uint32_t base = blockIdx.x * kBinRound; base < n; base += gridDim.x * kBinRound) {
      const uint32_t total = bin_round_setup<0>(rect, base, n, lrc, pre, wsum, s, [](int, uint32_t) {});
      __syncthreads();
      for (uint32_t j = tid; j < total; j += kBlock) {
        const int k = find_bin_item(pre, j);
        const uint32_t t = rect_tile(lrc[k], j - pre[k], s.tiles_x, s.rect_ys);
        if (!kBanded || t - t0 < nb) {
          const uint32_t slot = atomicSub(&hist[t - t0], 1u);
          if (slot < sb.bin_cap) bins[slot] = base + (uint32_t)k;
        }
      }
      __syncthreads();
    }
  }
}

// Exact range [xl, xr] (tile-local, clamped to [x0, x1]) of the pixels on row
// `ly` whose centres R covers.  Per edge, in tile-relative fixed point,
// E(lx) = c0 - dy*(256*lx + 128) with c0 = dx*(cy - ay) + dy*ax + bias exact
// (the spec's edge function with the top-left bias).  The boundary of each
// edge is solved in float (|error| << 1/16 px for a boundary near the tile);
// a 1/16-px margin makes the float range a superset of the covered pixels,
// larger by at most one pixel per side.  The covered set of a row is an
// interval (intersection of half-planes), so walking inward with the exact
// test until a covered pixel is found gives the exact range, and level-2
// fragments skip the test.  `Small` records (every vertex within 64 px of the
// tile origin) do the exact arithmetic in 32 bits with full-rate 24-bit
// multiplies; others in int64.
template <bool Small>
__device__ __forceinline__ void row_span(const uint4& g0, const uint4& g1, int ox, int oy, int ly, int x0, int x1,
                                         int& xl, int& xr, bool no_exact) {
  using T = typename std::conditional<Small, int32_t, int64_t>::type;
  const int32_t RX[3] = {(int32_t)g0.x, (int32_t)g0.y, (int32_t)g0.z};
  const int32_t RY[3] = {(int32_t)g0.w, (int32_t)g1.x, (int32_t)g1.y};
  const int32_t OX = ox * 256, OY = oy * 256;
  const int32_t cy = ly * 256 + 128;
  T c0[3];
  int32_t dys[3];
  float lo = -1.0e30f, hi = 1.0e30f;
  const int ea[3] = {1, 2, 0}, eb[3] = {2, 0, 1};
#pragma unroll
  for (int e = 0; e < 3; ++e) {
    const int32_t ax = RX[ea[e]] - OX, ay = RY[ea[e]] - OY;
    const int32_t dx = RX[eb[e]] - RX[ea[e]];
    const int32_t dy = RY[eb[e]] - RY[ea[e]];
    const int bias = (dy < 0 || (dy == 0 && dx > 0)) ? 0 : -1;
    if constexpr (Small) c0[e] = __mul24(dx, cy - ay) + __mul24(dy, ax) + bias;
    else c0[e] = (int64_t)dx * (cy - ay) + (int64_t)dy * ax + bias;
    dys[e] = dy;
    // boundary of the edge on this row, approximate (rcp: ~2 ulp, far below
    // the 1/16-px margin where it matters); branch-free (no divergence)
    const float t = (float)c0[e] * __builtin_amdgcn_rcpf((float)dy);
    hi = (dy > 0) ? fminf(hi, t) : hi;
    lo = (dy < 0) ? fmaxf(lo, t) : lo;
    hi = (dy == 0 && c0[e] < 0) ? -1.0e30f : hi;
  }
  // Near the strip the float boundaries are within ~1e-5 px of the exact ones
  // (tile-relative values below 2^14 units, ~2^-22 relative error).  An end
  // whose boundary lies farther than kEps from every pixel centre is exact as
  // computed: every left edge is at least kEps left of xl, every right edge at
  // least kEps right of xr.  Only a boundary within kEps of a centre (through
  // it: the top-left bias decides) is walked with the exact test.
  constexpr float kEps = 1.0f / 64.0f;
  const float lc = (lo - 128.0f) * (1.0f / 256.0f), hc = (hi - 128.0f) * (1.0f / 256.0f);
  const float lcc = fminf(fmaxf(lc, (float)x0 - 1.0f), (float)x1 + 1.0f);
  const float hcc = fmaxf(fminf(hc, (float)x1 + 1.0f), (float)x0 - 1.0f);
  xl = max((int)ceilf(lcc - kEps), x0);
  xr = min((int)floorf(hcc + kEps), x1);
  const float fl = lcc - floorf(lcc), fh = hcc - floorf(hcc);
  const bool walk_l = lc > (float)x0 - 0.5f && lc < (float)x1 + 0.5f && (fl <= kEps || fl >= 1.0f - kEps);
  const bool walk_r = hc > (float)x0 - 0.5f && hc < (float)x1 + 0.5f && (fh <= kEps || fh >= 1.0f - kEps);
  if (no_exact) return;   // ablation only (CSG_DEBUG 2048): superset span
  auto covers = [&](int lx) {
    const int32_t cx = lx * 256 + 128;
    bool in = true;
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      if constexpr (Small) in &= c0[e] - __mul24(dys[e], cx) >= 0;
      else in &= c0[e] - (int64_t)dys[e] * cx >= 0;
    }
    return in;
  };
  // normally zero or one step: keep the loops scalar (the loop vectorizer
  // otherwise evaluates eight speculative steps per trip)
  if (walk_l) {
#pragma clang loop vectorize(disable) interleave(disable) unroll(disable)
    while (xl <= xr && !covers(xl)) ++xl;
  }
  if (walk_r) {
#pragma clang loop vectorize(disable) interleave(disable) unroll(disable)
    while (xr >= xl && !covers(xr)) --xr;
  }
}

// ---------------------------------------------------------------------------
// k_raster: one 32x32 tile of one frame per 256-thread workgroup
// ---------------------------------------------------------------------------
// LDS image of up to kStage staged records as their five 16-B field groups (see
// Rec), group-major: lanes reading one group of different records hit
// consecutive 16-B slots (no bank conflicts; a record-strided image puts 8
// records on each set of banks), lanes reading the same record broadcast.
//
// Occupancy: k_raster is latency-bound (LDS and VMEM dependency chains), and
// waves per SIMD are its lever (measured on C3 against 4 waves: 3 waves +22%
// time, 5 waves -8%, 6 waves a further -5%; with 96-B records 7 waves a
// further -4%, 8 waves lose again to spills and small batches).  Seven
// 256-thread workgroups per CU need <= 22 KiB of LDS each (124 staged 80-B
// records, 116 shade-table slots) and <= 72 VGPRs.
// Per tile shape (workgroup size): 124 staged records / 116 shade slots for
// 256-thread workgroups (32 x 32), 64 / 64 for 128-thread ones (32 x 16; 56 /
// 60 / 64 staged: k_raster 98.6 / 97.0 / 96.2 ms per 2,880 frames, 64 is the
// most the LDS holds); either way 7 waves per SIMD fit the LDS and the 72-VGPR
// budget.
#ifndef CSG_STAGE
#define CSG_STAGE (kRasterBlock >= 256 ? 124 : 64)
#endif
#ifndef CSG_WAVES
#define CSG_WAVES 7             // k_raster waves per SIMD to budget registers for
#endif
#ifndef CSG_COV_STAGE          // k_raster<true>: smaller batches pay for the coverage table (7 waves per SIMD)
#define CSG_COV_STAGE (kRasterBlock >= 256 ? 72 : 38)
#endif
#ifndef CSG_COV_WAVES
#define CSG_COV_WAVES 7
#endif
#define CSG_RASTER_ATTR \
  __attribute__((amdgpu_waves_per_eu(kCov ? CSG_COV_WAVES : CSG_WAVES, kCov ? CSG_COV_WAVES : CSG_WAVES)))
constexpr int kStage = CSG_STAGE;     // records staged per raster batch (<= kRasterBlock)
static_assert(kStage <= kRasterBlock && CSG_COV_STAGE <= kRasterBlock, "one staged record per thread");
constexpr int kRB = kRasterBlock;
// level-2 items of one level-1 round: up to kRB spans of up to kTileW pixels,
// as 32-item words of the start bitmap
constexpr int kL2Words = kRB * kTileW / 32;
constexpr int kColWords = (kTileW + 31) / 32;   // 32-bit column masks per tile row (label statistics)
template <bool kCov>
constexpr int kStageOf = kCov ? CSG_COV_STAGE : kStage;
template <int NS>
struct RecImage {
  uint4 q[kRecGroups][NS];
};

// Coverage table of k_raster<true> (occlusion, GDP:1780-1790 occlusionRatio):
// for each label seen in the tile, the pixels some fragment of it covers
// (covered centre, depth in range, alpha test passed; no depth test), as a
// bit image of the tile (bit p & 31 of word p >> 5, p = ly * kTileW + lx).  A label that finds no slot (more than kCovSlots labels in
// one tile) marks the tile: its labels are then flagged unknown and their
// counts are not added, so the result does not depend on fragment order.
struct CovLds {
  uint32_t keys[kCovSlots];             // label of each slot (kNoAlpha: empty)
  uint32_t mask[kCovSlots][kTilePix / 32];   // per slot: the tile's pixels as bits
  uint32_t ovf;                         // some label found no slot
};

struct RasterCtx {
  const uint32_t* aquad;
  const uint32_t* acls;
  unsigned long long* zb;
  int ox, oy;
  float inv_near, inv_far;
  uint32_t dbg;
  uint32_t* ctr;   // profiling counters (CSG_DEBUG 512 only)
  CovLds* cov;     // k_raster<true> only
  int32_t* rlabel; // k_raster<true> only: label of each staged record (-1: not counted)
  uint32_t* gcov;  // covered[f][.] of this frame (k_raster<true> only)
};

// Mark pixel (lx, ly) covered by `label` in the tile's coverage table.
__device__ __forceinline__ void cov_mark(const RasterCtx& c, uint32_t label, int lx, int ly) {
  CovLds& t = *c.cov;
  const uint32_t h = label & (uint32_t)(kCovSlots - 1);
#pragma clang loop vectorize(disable) unroll(disable)
  for (uint32_t p = 0; p < (uint32_t)kCovSlots; ++p) {
    const uint32_t idx = (h + p) & (uint32_t)(kCovSlots - 1);
    uint32_t cur = t.keys[idx];
    if (cur == kNoAlpha) cur = atomicCAS(&t.keys[idx], kNoAlpha, label);
    if (cur == kNoAlpha || cur == label) {
      const uint32_t px = (uint32_t)(ly * kTileW + lx);
      atomicOr(&t.mask[idx][px >> 5], 1u << (px & 31u));
      return;
    }
  }
  t.ovf = 1u;
  atomicOr(&c.gcov[label], kCovUnknown);
}

// Slot of `label` in the coverage table, or -1 if it has none yet (read-only
// probe).  Slots are never freed and fill in probe order, so an empty slot
// ends the search; a slot taken concurrently reads as "none", which only
// sends the fragment to cov_mark.
__device__ __forceinline__ int cov_find(const RasterCtx& c, uint32_t label) {
  const CovLds& t = *c.cov;
  const uint32_t h = label & (uint32_t)(kCovSlots - 1);
#pragma clang loop vectorize(disable) unroll(disable)
  for (uint32_t p = 0; p < (uint32_t)kCovSlots; ++p) {
    const uint32_t idx = (h + p) & (uint32_t)(kCovSlots - 1);
    const uint32_t cur = t.keys[idx];
    if (cur == label) return (int)idx;
    if (cur == kNoAlpha) return -1;
  }
  return -1;
}


__device__ __forceinline__ float f_(uint32_t u) { return __uint_as_float(u); }

// Z-buffer word of tile pixel (lx, ly): row-major with the column XORed by
// the row (CSG_ZB_SWIZZLE).  A row-major tile of 8-B words puts every row on
// the same LDS banks, so fragments at one column of a stack of rows (a small
// record's rows, vertically aligned spans) and the resolve's 4-pixel groups
// (lanes t and t+8 of a lane group 32 B x 8 apart) met on one bank pair
// (profiles/r05/ab/lds_counters.txt).  XORing the column with the row keeps
// each row a permutation of its words (consecutive pixels of a span stay
// distinct) and each aligned 4-pixel group inside its own 32 B.
#ifndef CSG_ZB_SWIZZLE
#define CSG_ZB_SWIZZLE 1
#endif
__device__ __forceinline__ int zb_index(int lx, int ly) {
  return ly * kTileW + (CSG_ZB_SWIZZLE ? (lx ^ (ly & (kTileW - 1))) : lx);
}

// One fragment of staged record k at tile pixel (lx, ly), already known to be
// covered: homogeneous depth, depth range, early-z against the LDS key,
// alpha test (texture described inline in the record), then ds_min_u64.
// With kCov (occlusion) every fragment in the depth range is alpha-tested,
// early-z or not, and a surviving one marks its label's coverage bit.
template <bool kCov, int NS>
__device__ __forceinline__ void fragment(const RasterCtx& c, const RecImage<NS>& I, int k, int lx, int ly) {
  const float fx = (float)(c.ox + lx) + 0.5f, fy = (float)(c.oy + ly) + 0.5f;
  const uint4 g2 = I.q[2][k], g4 = I.q[4][k];
  const float invw = plane_at(f_(g2.z), f_(g2.w), f_(g4.z), fx, fy);
  if (!(invw >= c.inv_far && invw <= c.inv_near)) return;
  // alpha test at the pixel centre: u = U(x, y) * (1 / (1/W)), v likewise;
  // both planes at once in packed FP32, per component ((U0*x + U1*y) + U2) * r
  auto alpha_ok = [&]() {
    const uint4 g3 = I.q[3][k];
    const float r = rcp_ieee(invw);   // invw in [1/far, 1/near]
    const f32x2 p0 = {f_(g3.x), f_(g3.y)}, p1 = {f_(g3.z), f_(g3.w)}, p2 = {f_(g4.x), f_(g4.y)};
    const f32x2 uv = ((p0 * fx + p1 * fy) + p2) * r;
    return alpha_pass(c.aquad, c.acls, (g2.y & 0xFFFFFFu) * kTexAlign, g4.w, (int)(g2.y >> 24), uv.x, uv.y);
  };
  const unsigned long long key = ((unsigned long long)(0xFFFFFFFFu - fbits(invw)) << 32) | g2.x;
  unsigned long long* z = &c.zb[zb_index(lx, ly)];
  if constexpr (kCov) {
    // A fragment has two possible effects: its label's coverage bit and the
    // depth minimum.  One that loses early-z and whose bit is already set has
    // neither, so it skips the alpha test (both are monotone: a stale read only
    // sends a fragment down the full path).
    const int32_t lab = c.rlabel[k];
    const bool zwin = key < *z;
    int slot = -1;
    bool mark = false;
    if (lab >= 0) {
      slot = cov_find(c, (uint32_t)lab);
      const uint32_t px = (uint32_t)(ly * kTileW + lx);
      mark = slot < 0 || !((c.cov->mask[slot][px >> 5] >> (px & 31u)) & 1u);
    }
    if (!zwin && !mark) return;
    if (g2.y != kNoAlpha && !alpha_ok()) return;
    if (mark) {
      if (slot >= 0) {
        const uint32_t px = (uint32_t)(ly * kTileW + lx);
        atomicOr(&c.cov->mask[slot][px >> 5], 1u << (px & 31u));
      }
      else cov_mark(c, (uint32_t)lab, lx, ly);
    }
    if (zwin) atomicMin(z, key);
    return;
  }
  // Without an alpha test the ds_min_u64 is the depth test: no early-z read,
  // compare and branch (a losing key leaves the word unchanged).
  if (g2.y == kNoAlpha && !(DBG(c.dbg) & 512u)) {
    atomicMin(z, key);
    return;
  }
  if (!(DBG(c.dbg) & 16u) && key >= *z) {
    if (DBG(c.dbg) & 512u) atomicAdd(&c.ctr[7], 1u);   // profiling: early-z rejects
    return;
  }
  if (!(DBG(c.dbg) & 4u) && g2.y != kNoAlpha) {
    if (DBG(c.dbg) & 512u) {   // profiling: wave executions of the alpha test and their active lanes
      const uint64_t m = __ballot(1);
      if ((uint32_t)__lane_id() == (uint32_t)__ffsll((unsigned long long)m) - 1u) {
        atomicAdd(&c.ctr[12], 1u);
        atomicAdd(&c.ctr[13], (uint32_t)__popcll(m));
      }
    }
    const bool pass = alpha_ok();
    if (DBG(c.dbg) & 512u) atomicAdd(&c.ctr[pass ? 6 : 5], 1u);   // profiling: alpha tests passed / failed
    if (!pass) return;
  }
  atomicMin(z, key);
}

// Stage bin entry `idx` into `slot`; returns its row count inside the tile.
template <int NS>
__device__ __forceinline__ uint32_t stage_record_r(const Rec* recs, uint32_t r, uint32_t rec_cap, RecImage<NS>& img,
                                                   int slot, int ox, int oy, uint32_t& row0);
template <int NS>
__device__ __forceinline__ uint32_t stage_record(const Rec* recs, const uint32_t* bins, uint32_t idx, uint32_t end,
                                                 uint32_t rec_cap, RecImage<NS>& img, int slot, int ox, int oy,
                                                 uint32_t& row0) {
  const uint32_t r = (idx < end && slot < NS) ? bins[idx] : 0xFFFFFFFFu;
  return stage_record_r<NS>(recs, r, rec_cap, img, slot, ox, oy, row0);
}
// ... with the record id `r` already loaded (kNoRecord: none)
template <int NS>
__device__ __forceinline__ uint32_t stage_record_r(const Rec* recs, uint32_t r, uint32_t rec_cap, RecImage<NS>& img,
                                                   int slot, int ox, int oy, uint32_t& row0) {
  row0 = 0;
  if (r >= rec_cap) return 0;
  const uint4* src = reinterpret_cast<const uint4*>(recs + r);
  uint4 q[kRecGroups];
#pragma unroll
  for (int k = 0; k < kRecGroups; ++k) q[k] = src[k];
#pragma unroll
  for (int k = 0; k < kRecGroups; ++k) img.q[k][slot] = q[k];
  const uint32_t p0 = q[1].z, p1 = q[1].w;            // px0 | py0 << 16, px1 | py1 << 16
  int y0 = max((int)(p0 >> 16), oy), y1 = min((int)(p1 >> 16), oy + kTileH - 1);
  const int x0 = max((int)(p0 & 0xFFFFu), ox), x1 = min((int)(p1 & 0xFFFFu), ox + kTileW - 1);
  if (x0 > x1 || y0 > y1) return 0u;
  // Rows of the triangle inside this tile's column strip: the y-range of the
  // triangle clipped to the pixel-centre lines x0..x1, in float relative to
  // the tile, widened by half a pixel (>> any rounding here); the exact row
  // spans of level 1 decide coverage, this only drops rows that cannot have any.
  const int32_t X[3] = {(int32_t)q[0].x, (int32_t)q[0].y, (int32_t)q[0].z};
  const int32_t Y[3] = {(int32_t)q[0].w, (int32_t)q[1].x, (int32_t)q[1].y};
  const float sl = (float)(x0 * 256 + 128), sr = (float)(x1 * 256 + 128);
  float fx[3], fy[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) { fx[k] = (float)X[k]; fy[k] = (float)(Y[k] - oy * 256); }
  float ylo = 1.0e30f, yhi = -1.0e30f;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    if (fx[k] >= sl && fx[k] <= sr) { ylo = fminf(ylo, fy[k]); yhi = fmaxf(yhi, fy[k]); }
    const int n = (k + 1) % 3;
    const float dxe = fx[n] - fx[k], dye = fy[n] - fy[k];
    // 1/dxe: hardware reciprocal + one Newton step (<= ~1 ulp; the half-pixel
    // widening below covers it), instead of two IEEE divisions per edge
    const float r0 = __builtin_amdgcn_rcpf(dxe);
    const float rdx = fmaf(fmaf(-dxe, r0, 1.0f), r0, r0);
#pragma unroll
    for (int side = 0; side < 2; ++side) {
      const float xs = side ? sr : sl;
      if ((fx[k] - xs) * (fx[n] - xs) < 0.0f) {
        const float yc = fy[k] + (xs - fx[k]) * rdx * dye;
        ylo = fminf(ylo, yc);
        yhi = fmaxf(yhi, yc);
      }
    }
  }
  bool small = true;
#pragma unroll
  for (int k = 0; k < 3; ++k)
    small &= abs(X[k] - ox * 256) < (1 << 14) && abs(Y[k] - oy * 256) < (1 << 14);
  if (!(ylo <= yhi)) return 0u;
  // Vertices within 64 px of the tile: every value above is below 2^16 units
  // and off by < 0.01 units, so a 1/16-px widening suffices (half a pixel
  // otherwise added about one empty row per record and tile).
  const float wid = small ? 16.0f : 128.0f;
  const int r0 = (int)ceilf((ylo - 128.0f - wid) * (1.0f / 256.0f));
  const int r1 = (int)floorf((yhi - 128.0f + wid) * (1.0f / 256.0f));
  y0 = max(y0, oy + r0);
  y1 = min(y1, oy + r1);
  row0 = (uint32_t)(y0 - oy) | (small ? 0x80u : 0u);
  return y0 <= y1 ? (uint32_t)(y1 - y0 + 1) : 0u;
}

// Software-pipelined staging (round 6): a batch's bin entries (record ids)
// are loaded one batch ahead -- the first batch's by k_raster before the
// z-buffer initialisation, each later batch's right after the previous batch's
// records -- so a batch's staging waits for one dependent global load (the
// record) instead of two (bin entry, then record).  Staging was 92% parked
// wave-cycles.  Measured on C3 at 2,880 frames per launch, 3 runs
// each: k_raster 96.4 -> 93.8 ms, frames/s +2.3%, 72 VGPRs either way
// (profiles/r06/ab/raster_variants_F2880.txt).  CSG_PREFETCH_BIN=0 builds the
// previous staging for A/B.
#ifndef CSG_PREFETCH_BIN
#define CSG_PREFETCH_BIN 1
#endif

template <int NS>
struct RasterLds {
  RecImage<NS> img;                     // staged bin records
  uint32_t starts1[NS];                 // bit i: a staged record's rows start at level-1 item i
  uint16_t before1[NS + 1];             // records starting before item 32*d
  uint32_t crec[NS];                    // compact record: slot | first item << 8
  uint8_t row0[NS];                     // first tile row of each staged record | 0x80 if small
  uint32_t span[kRB];                   // rec | ly << 8 | (ex2 - xl + kTileW) << 16
  uint32_t starts[kL2Words];            // bit i: a span starts at level-2 item i (<= kRB spans x kTileW px)
  uint16_t before[kL2Words + 1];        // spans starting before item 32*d
  uint32_t wsum[kRB / 64];              // the batch scan's wave totals
  uint32_t wsum2[kRB / 64];             // the level-2 scan's (each reused only after other barriers)
};

// Block-level two-level expansion of kStage-record batches.
//   level 1: (record, row) items, one per thread -> exact row span
//   level 2: (span, pixel) items
// An item finds its record / span by a rank query over a bitmap of starts
// (measured: -5.5% k_raster vs a 4-ary search over the prefix; a per-item
// owner map cost a workgroup per CU in LDS).
template <bool kCov, int NS>
__device__ __forceinline__ void raster_block(const RasterCtx& c, const SceneDev& s, const BatchDev& b, RasterLds<NS>& L,
                                             uint32_t beg, uint32_t end, const uint32_t* bins, const Rec* recs,
                                             uint32_t rec_cap, uint32_t rfirst) {
  const int tid = threadIdx.x;
#if CSG_PREFETCH_BIN
  // software-pipelined staging: each batch's record ids are loaded one batch
  // ahead (issued after the current batch's records, consumed by the next
  // batch; the first batch's by k_raster before the z-buffer initialisation),
  // so a batch's staging waits for one dependent load, not two
  uint32_t rnext = rfirst;
#endif
  for (uint32_t base = beg; base < end; base += NS) {
    uint32_t row0;
#if CSG_PREFETCH_BIN
    const uint32_t rows = stage_record_r<NS>(recs, rnext, rec_cap, L.img, tid, c.ox, c.oy, row0);
    rnext = (tid < NS && base + NS + (uint32_t)tid < end) ? bins[base + NS + tid] : 0xFFFFFFFFu;
#else
    const uint32_t rows = stage_record(recs, bins, base + tid, end, rec_cap, L.img, tid, c.ox, c.oy, row0);
#endif
    if (tid < NS) L.row0[tid] = (uint8_t)row0;
    if constexpr (kCov) {   // label of the staged record (read back from this thread's own slot)
      if (tid < NS) {
        int32_t lab = -1;
        if (rows) {
          lab = s.inst[L.img.q[2][tid].x >> s.uid_shift].label;
          if (lab >= 0 && (uint32_t)lab >= b.n_labels) lab = -1;
        }
        c.rlabel[tid] = lab;
      }
    }
    if ((DBG(b.dbg) & 512u) && rows) {   // profiling counters: records with rows in the tile, row items
      atomicAdd(&b.overflow[1], 1u);
      atomicAdd(&b.overflow[2], rows);
      const uint4 g1 = L.img.q[1][tid];
      if (((g1.w & 0xFFFFu) - (g1.z & 0xFFFFu)) < 4u && ((g1.w >> 16) - (g1.z >> 16)) < 4u) {
        atomicAdd(&b.overflow[9], 1u);      // records whose pixel box is at most 4 x 4
        atomicAdd(&b.overflow[10], rows);   // ... their row items
      }
    }
    // records with rows get compact indices; item -> record is a rank query
    // over a bitmap of record starts (as for level 2 below)
    if (tid < NS) L.starts1[tid] = 0u;   // ordered before the atomics by the scan's barriers
    if (tid == 0) L.before1[0] = 0;
    uint32_t tot1p;
    const uint32_t ex1p = block_excl_scan<false, kRB>(rows | (rows ? 0x10000u : 0u), L.wsum, tot1p);
    const uint32_t tot1 = tot1p & 0xFFFFu;
    if (rows) {
      const uint32_t ex1 = ex1p & 0xFFFFu, ci = ex1p >> 16, e_end = ex1 + rows;
      L.crec[ci] = (uint32_t)tid | (ex1 << 8);
      atomicOr(&L.starts1[ex1 >> 5], 1u << (ex1 & 31u));
      if ((e_end & ~31u) > ex1) L.before1[e_end >> 5] = (uint16_t)(ci + 1u);
    }
    __syncthreads();
    for (uint32_t c1 = 0; c1 < ((DBG(b.dbg) & 256u) ? 0u : tot1); c1 += kRB) {
      const uint32_t j1 = c1 + tid;
      uint32_t w2 = 0, sp = 0;
      int xl = 0;
      if (j1 < tot1) {
        const uint32_t w1 = L.starts1[j1 >> 5], nb1 = L.before1[j1 >> 5];
        const uint32_t cr = L.crec[nb1 + (uint32_t)__popc(w1 & (0xFFFFFFFFu >> (31u - (j1 & 31u)))) - 1u];
        const int k = (int)(cr & 255u);
        const uint32_t first = cr >> 8;
        const uint4 g0 = L.img.q[0][k], g1 = L.img.q[1][k];
        const int x0 = max((int)(g1.z & 0xFFFFu) - c.ox, 0), x1 = min((int)(g1.w & 0xFFFFu) - c.ox, kTileW - 1);
        const uint32_t r0b = L.row0[k];
        const int ly = (int)(r0b & 31u) + (int)(j1 - first);
        int xr;
        if (DBG(b.dbg) & 1024u) { xl = 1; xr = 0; }   // ablation: no span computation
        else if (r0b & 0x80u) row_span<true>(g0, g1, c.ox, c.oy, ly, x0, x1, xl, xr, DBG(b.dbg) & 2048u);
        else {
          if (DBG(b.dbg) & 512u) atomicAdd(&b.overflow[8], 1u);   // profiling: row items on the int64 path
          row_span<false>(g0, g1, c.ox, c.oy, ly, x0, x1, xl, xr, DBG(b.dbg) & 2048u);
        }
        if (xl <= xr) {
          w2 = (uint32_t)(xr - xl + 1);
          sp = (uint32_t)k | ((uint32_t)ly << 8);
        }
      }
      if ((DBG(b.dbg) & 512u) && w2) {      // non-empty spans, level-2 items
        atomicAdd(&b.overflow[3], 1u);
        atomicAdd(&b.overflow[4], w2);
        const uint4 g1 = L.img.q[1][sp & 255u];
        if (((g1.w & 0xFFFFu) - (g1.z & 0xFFFFu)) < 4u && ((g1.w >> 16) - (g1.z >> 16)) < 4u)
          atomicAdd(&b.overflow[11], w2);   // level-2 items of records with at most 4 x 4 box
      }
      // Non-empty spans get compact indices (one packed scan gives item
      // offset and index).  Item -> span is then a rank query: a bitmap of
      // span starts plus, per 32-item word, the spans starting before it (the
      // one span crossing each word boundary writes it) -- two independent
      // LDS reads and a popcount instead of a 4-step search.
      // zeroed before the atomics below (ordered by the scan's barriers)
      if constexpr (kL2Words >= kRB) {
#pragma unroll
        for (int w = 0; w < kL2Words / kRB; ++w) L.starts[tid + w * kRB] = 0u;
      } else if (tid < kL2Words) {
        L.starts[tid] = 0u;
      }
      if (tid == 0) L.before[0] = 0;
      uint32_t totp;
      const uint32_t exp = block_excl_scan<false, kRB>(w2 | (w2 ? 0x10000u : 0u), L.wsum2, totp);
      const uint32_t ex2 = exp & 0xFFFFu, tot2 = totp & 0xFFFFu;
      if (w2) {
        const uint32_t ci = exp >> 16, e_end = ex2 + w2;
        L.span[ci] = sp | ((ex2 - (uint32_t)xl + (uint32_t)kTileW) << 16);
        atomicOr(&L.starts[ex2 >> 5], 1u << (ex2 & 31u));
        // the spans starting before each 32-item word boundary inside (ex2, e_end]
        // (a span of <= 32 items crosses at most one)
        if constexpr (kTileW <= 32) {
          if ((e_end & ~31u) > ex2) L.before[e_end >> 5] = (uint16_t)(ci + 1u);
        } else {
          for (uint32_t d = (ex2 >> 5) + 1u; d <= (e_end >> 5); ++d) L.before[d] = (uint16_t)(ci + 1u);
        }
      }
      __syncthreads();
      for (uint32_t j = tid; j < ((DBG(b.dbg) & 8u) ? 0u : tot2); j += kRB) {
        if (DBG(b.dbg) & 512u) {   // profiling: level-2 wave iterations and their active lanes
          const uint64_t m = __ballot(1);
          if ((uint32_t)__lane_id() == (uint32_t)__ffsll((unsigned long long)m) - 1u) {
            atomicAdd(&b.overflow[14], 1u);
            atomicAdd(&b.overflow[15], (uint32_t)__popcll(m));
          }
        }
        const uint32_t w = L.starts[j >> 5], nb = L.before[j >> 5];
        const uint32_t rank = nb + (uint32_t)__popc(w & (0xFFFFFFFFu >> (31u - (j & 31u))));
        const uint32_t spj = L.span[rank - 1u];
        fragment<kCov>(c, L.img, (int)(spj & 255u), (int)(j + (uint32_t)kTileW - (spj >> 16)), (int)((spj >> 8) & 255u));
      }
      __syncthreads();
    }
  }
}

// ---------------------------------------------------------------------------
// per-pixel resolve
// ---------------------------------------------------------------------------
// Everything the resolve needs about one winning triangle (84 B).  P holds the
// homogeneous edge rows A0-2 B0-2 C0-2, invdet and the uvs while the entry is
// set up, then the screen planes D0-2 U0-2 V0-2 of 1/W, u/W, v/W (spec
// §3.5-6; U, V for textured triangles only).
struct ShadeEntry {
  float P[16];
  int32_t label;
  int32_t tex;                      // -1: flat albedo
  uint32_t base;                    // albedo multiplier r | g << 8 | b << 16
  uint32_t q01, q2;                 // shade factors (x256): q0 | q1 << 16, q2
  uint32_t n01, n2;                 // unit world normal facing the camera, f16: x | y << 16, z
};

// Triangle setup of the resolve, exactly as csg_oracle.c: clip coordinates,
// homogeneous coefficients, material, uvs, flat two-sided Lambert from the
// world-space face normal.
// `e` is the triangle's LDS slot: fields are stored as soon as they are
// known, and the clip and model rows are consumed one at a time, so few
// values are live at once (this phase sets the kernel's register budget).
__device__ __forceinline__ void shade_setup(const SceneDev& s, const BatchDev& b, uint32_t f, uint32_t uid,
                                            ShadeEntry& e) {
  const uint32_t i = uid >> s.uid_shift, g = uid & ((1u << s.uid_shift) - 1u);   // instance, soup index
  const uint32_t set = b.fset[f];
  const float* tp = s.tri_pos + (size_t)g * 9;
  float p[9];
#pragma unroll
  for (int z = 0; z < 9; ++z) p[z] = tp[z];
  const InstSetDev is = b.iset[(size_t)set * s.n_inst + i];   // (independent of the triangle loads)
  e.label = is.label;
  const int tex = is.tex;
  e.tex = tex;
  e.base = is.base;
  const float* tu = s.tri_uv + (size_t)g * 6;
#pragma unroll
  for (int z = 0; z < 6; ++z) e.P[10 + z] = tex >= 0 ? tu[z] : 0.0f;
  // Homogeneous coefficients: for texture coordinates, depth / points and the
  // normals' facing sign only (a flat-shaded triangle without those outputs
  // needs none of them: no clip transform, no IEEE reciprocal).
  bool facing = false;
  if (tex >= 0 || b.depth || b.points || b.normals) {
    Cv3 v[3];
    const float* Cm = b.clip + ((size_t)f * s.n_inst + i) * 12;
#pragma unroll
    for (int z = 0; z < 3; ++z) {
      v[z].x = dot4(Cm + 0, p[3 * z], p[3 * z + 1], p[3 * z + 2]);
      v[z].y = dot4(Cm + 4, p[3 * z], p[3 * z + 1], p[3 * z + 2]);
      v[z].w = dot4(Cm + 8, p[3 * z], p[3 * z + 1], p[3 * z + 2]);
    }
    Hom h;
    hom_setup(v, h);
#pragma unroll
    for (int z = 0; z < 3; ++z) { e.P[z] = h.A[z]; e.P[3 + z] = h.B[z]; e.P[6 + z] = h.C[z]; }
    e.P[9] = h.invdet;
    facing = h.invdet < 0.0f;
  }
  // world-space edges e1 = pw1 - pw0, e2 = pw2 - pw0, one model row (= one
  // world coordinate) at a time
  float e1[3], e2[3];
  {
    const float* M = b.models + ((size_t)set * s.n_inst + i) * 16;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const float w0 = dot4(M + 4 * r, p[0], p[1], p[2]);
      const float w1 = dot4(M + 4 * r, p[3], p[4], p[5]);
      const float w2 = dot4(M + 4 * r, p[6], p[7], p[8]);
      e1[r] = w1 - w0;
      e2[r] = w2 - w0;
    }
  }
  const float nx = e1[1] * e2[2] - e1[2] * e2[1];
  const float ny = e1[2] * e2[0] - e1[0] * e2[2];
  const float nz = e1[0] * e2[1] - e1[1] * e2[0];
  const float nn = (nx * nx + ny * ny) + nz * nz;
  const LightDev& L = b.lights[set];
  float cs = 0.0f;
  uint32_t n01 = 0, n2 = 0;
  if (nn > 0.0f) {
    const float len = sqrtf(nn);
    const float d = (nx * L.sun_dir[0] + ny * L.sun_dir[1]) + nz * L.sun_dir[2];
    cs = fabsf(d / len);
    // two-sided: the clip-space determinant is negative exactly when the face
    // normal points toward the camera (pixel projection with fx*fy > 0)
    if (b.normals) {   // (three IEEE divisions: only when normals are an output)
      const float sg = facing ? 1.0f : -1.0f;
      n01 = half_bits(sg * (nx / len)) | (half_bits(sg * (ny / len)) << 16);
      n2 = half_bits(sg * (nz / len));
    }
  }
  e.n01 = n01;
  e.n2 = n2;
  uint32_t q[3];
#pragma unroll
  for (int z = 0; z < 3; ++z) {
    const float shade = L.ambient[z] + L.sun[z] * cs;
    const int qq = (int)(shade * 256.0f + 0.5f);
    q[z] = (uint32_t)min(max(qq, 0), 65535);
  }
  e.q01 = q[0] | (q[1] << 16);
  e.q2 = q[2];
  // The planes, from the entry's LDS copy: a separate phase, so the edge rows
  // and uvs are not all live in registers together with the setup's state.
  __asm__ volatile("" ::: "memory");
  float P[16];
#pragma unroll
  for (int z = 0; z < 16; ++z) P[z] = e.P[z];
  float D[3], U[3], V[3];
  depth_plane(P, P + 3, P + 6, P[9], D);
  uv_planes(P, P + 3, P + 6, P[9], P + 10, U, V);
  // D in P[0..2]; the u and v planes as aligned (U_k, V_k) pairs in P[4..9]
  // for shade_pixel's packed evaluation
#pragma unroll
  for (int z = 0; z < 3; ++z) { e.P[z] = D[z]; e.P[4 + 2 * z] = U[z]; e.P[5 + 2 * z] = V[z]; }
}

// Depth, instance id and RGB of pixel (px, py) covered by entry e.
// The homogeneous evaluation is needed only for the depth (when depth or
// points are requested) and for texture coordinates.
__device__ __forceinline__ void shade_pixel(const SceneDev& s, const ShadeEntry& e, int px, int py, bool need_depth,
                                            uint32_t& rgb_out, int32_t& id_out, float& depth_out) {
  const bool textured = e.tex >= 0 && !(DBG(s.dbg) & 4096u);   // 4096: ablation only, no texture fetch
  const float fx = (float)px + 0.5f, fy = (float)py + 0.5f;
  float r = INFINITY;
  if (need_depth || textured) r = rcp_ieee(plane_at(e.P[0], e.P[1], e.P[2], fx, fy));   // the winner's invW
  depth_out = need_depth ? r : INFINITY;
  id_out = e.label;
  int base[3] = {(int)(e.base & 255u), (int)((e.base >> 8) & 255u), (int)((e.base >> 16) & 255u)};
  int alb[3];
  if (textured) {   // u, v in packed FP32, per component ((U0*x + U1*y) + U2) * r
    const f32x2 p0 = {e.P[4], e.P[5]}, p1 = {e.P[6], e.P[7]}, p2 = {e.P[8], e.P[9]};
    const f32x2 uv = ((p0 * fx + p1 * fy) + p2) * r;
    int c[4];
    tex_sample(s, e.tex, uv.x, uv.y, c);
#pragma unroll
    for (int z = 0; z < 3; ++z) alb[z] = div255(__umul24((uint32_t)c[z], (uint32_t)base[z]) + 127u);
  } else {
#pragma unroll
    for (int z = 0; z < 3; ++z) alb[z] = base[z];
  }
  const int q[3] = {(int)(e.q01 & 0xFFFFu), (int)(e.q01 >> 16), (int)e.q2};
  uint32_t o = 0;
#pragma unroll
  for (int z = 0; z < 3; ++z) o |= (uint32_t)min((int)((__umul24((uint32_t)alb[z], (uint32_t)q[z]) + 128u) >> 8), 255) << (8 * z);
  rgb_out = o;
}

#ifndef CSG_VEC_OUT
#define CSG_VEC_OUT 1      // vector stores of the per-pixel outputs (see the resolve)
#endif
#ifndef CSG_VEC_DEP_ONCE
#define CSG_VEC_DEP_ONCE 1 // a vector group's shading loop skips the depth (C5 k_raster -0.3%)
#endif

// Resolve-phase LDS (aliases the raster loop's): the tile's distinct winning
// triangles in an open-addressing table of kShadeSlots, each set up once by
// one thread, then read by every pixel that shows it.
#ifndef CSG_SHADE_SLOTS
#define CSG_SHADE_SLOTS (kRasterBlock >= 256 ? 116 : 64)
#endif
constexpr uint32_t kShadeSlots = CSG_SHADE_SLOTS;   // <= kRasterBlock (one setup thread per slot)
static_assert(kShadeSlots <= (uint32_t)kRasterBlock && kShadeSlots < 255u, "one setup thread per slot; 8-bit slot ids");
constexpr int kShadeProbes = 16;
struct ResolveLds {
  uint32_t keys[kShadeSlots];       // uid or kNoAlpha (empty)
  uint32_t more;                    // a pixel is left for another round
  ShadeEntry tab[kShadeSlots];
  uint32_t lstat[2 + kColWords][kMaxLdsLabels];   // per label: pixel count, row mask, column mask(s) (tile-relative bits)
};

// The resolve's LDS aliases the raster loop's in a union inside k_raster.
// (Measured with 4-wave workgroups: 31,776 B per workgroup keeps 5 per CU,
// 32,512 B gave 4; 26,656 B keeps 6; 22,448 B keeps 7.)  Other workgroup
// sizes (tile shapes): the same 160 KiB per CU less the 4-wave table's
// observed slack, shared by waves * 4 / (waves per workgroup) workgroups.
constexpr size_t lds_budget(int waves) {
  return kRasterBlock == 256
             ? (waves >= 8 ? 20480u : waves == 7 ? 22528u : waves == 6 ? 26700u : waves == 5 ? 32256u : 40960u)
             : ((157696u / (size_t)(waves * 4 / (kRasterBlock / 64))) & ~511u);
}
static_assert((sizeof(RasterLds<kStage>) > sizeof(ResolveLds) ? sizeof(RasterLds<kStage>) : sizeof(ResolveLds)) +
                      kTilePix * 8 <= lds_budget(CSG_WAVES),
              "k_raster LDS must allow CSG_WAVES workgroups per CU");

// The raster loop's side of the union; k_raster<true> adds the coverage table
// (it is flushed before the resolve starts, so the resolve may reuse it).
template <bool kCov>
struct RasterSide {
  RasterLds<kStageOf<kCov>> r;
};
template <>
struct RasterSide<true> {
  RasterLds<kStageOf<true>> r;
  CovLds cov;
  int32_t rlabel[kStageOf<true>];       // label of each staged record (-1: not counted)
};
static_assert((sizeof(RasterSide<true>) > sizeof(ResolveLds) ? sizeof(RasterSide<true>) : sizeof(ResolveLds)) +
                      kTilePix * 8 <= lds_budget(CSG_COV_WAVES),
              "k_raster<true> LDS must allow CSG_COV_WAVES workgroups per CU");

// Slot of `uid` in the table (inserting it), or -1 if the probe run is full.
__device__ __forceinline__ int shade_slot(uint32_t* keys, uint32_t uid) {
  const uint32_t h = __umulhi(uid * 2654435761u, kShadeSlots);   // [0, kShadeSlots)
#pragma clang loop vectorize(disable) unroll(disable)
  for (int p = 0; p < kShadeProbes; ++p) {
    uint32_t idx = h + (uint32_t)p;
    idx = idx >= kShadeSlots ? idx - kShadeSlots : idx;
    const uint32_t prev = atomicCAS(&keys[idx], kNoAlpha, uid);
    if (prev == kNoAlpha || prev == uid) return (int)idx;
  }
  return -1;
}

// XCD-aware tile order.  Workgroups are dealt round-robin over the 8 XCDs, so
// blocks v and v + 8 share an L2.  Each run of 32 blocks covers 8 squares of
// 2x2 tiles (squares in raster order), one square per XCD: the 4 tiles of a
// square share one L2, so a record binned to several of them is fetched once,
// while all XCDs keep working side by side on the same part of the frame.
// Blocks past the frame's edge (odd tile counts) return at once.
#ifndef CSG_SQ_X
#define CSG_SQ_X 2
#endif
#ifndef CSG_SQ_Y
#define CSG_SQ_Y 2
#endif
constexpr uint32_t kSqX = CSG_SQ_X, kSqY = CSG_SQ_Y;   // a square's edge in tiles (x, y)
constexpr uint32_t kSqN = kSqX * kSqY;
__device__ __forceinline__ bool swizzled_tile(uint32_t v, uint32_t tiles_x, uint32_t tiles_y, uint32_t& tile) {
  const uint32_t sqx = (tiles_x + kSqX - 1) / kSqX, sqy = (tiles_y + kSqY - 1) / kSqY;
  const uint32_t sq = (v / (8u * kSqN)) * 8u + (v & 7u), j = (v >> 3) % kSqN;
  if (sq >= sqx * sqy) return false;
  const uint32_t tx = (sq % sqx) * kSqX + (j % kSqX), ty = (sq / sqx) * kSqY + (j / kSqX);
  if (tx >= tiles_x || ty >= tiles_y) return false;
  tile = ty * tiles_x + tx;
  return true;
}

// Output stores of 4 consecutive pixels (a thread's quarter of a tile row).
// ids: 16 B, and 8 threads write a tile row's ids as one aligned 128-B line,
// stored non-temporally (kept out of L2, where records and textures are
// re-read; C3: raster -0.2%, profiles/r03/ab/output_stores.txt); RGB8: 12 B as
// one 3-dword store (4-B aligned: the pixel index is a multiple of 4; its
// 96-B row segments are not whole lines, so they stay ordinary stores).
typedef int32_t v4i32 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void out_ids(int32_t* p, int4 v) {
  const v4i32 w = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(w, reinterpret_cast<v4i32*>(p));
}
// The optional per-pixel outputs as 16-B / 8-B vector stores, non-temporal
// as the instance ids (CSG_NT_OUT; outputs are written once and never read
// back, so they need not displace records and texels from L2: C5 k_raster
// 66.4 -> 62.2 ms per 480 frames, profiles/r05/ab/tile_shape.md §10).
#ifndef CSG_NT_OUT
#define CSG_NT_OUT 1
#endif
#ifndef CSG_NT_RGB
#define CSG_NT_RGB 1      // the RGB group stores too (C3 k_raster 96.25 -> 95.86 ms, tile_shape.md §10)
#endif
typedef uint32_t v3u32 __attribute__((ext_vector_type(3)));
typedef float v4f32 __attribute__((ext_vector_type(4)));
typedef uint32_t v2u32 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void out_f4(float* p, float a, float b2, float c, float d) {
  const v4f32 w = {a, b2, c, d};
  if (CSG_NT_OUT) __builtin_nontemporal_store(w, reinterpret_cast<v4f32*>(p));
  else *reinterpret_cast<v4f32*>(p) = w;
}
__device__ __forceinline__ void out_u2(uint16_t* p, uint32_t a, uint32_t b2) {
  const v2u32 w = {a, b2};
  if (CSG_NT_OUT) __builtin_nontemporal_store(w, reinterpret_cast<v2u32*>(p));
  else *reinterpret_cast<v2u32*>(p) = w;
}
__device__ __forceinline__ void out_rgb4(uint8_t* p, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3) {
  const v3u32 w = {c0 | (c1 << 24), (c1 >> 8) | (c2 << 16), (c2 >> 16) | (c3 << 8)};
  if (CSG_NT_RGB) __builtin_nontemporal_store(w, reinterpret_cast<v3u32*>(p));
  else *reinterpret_cast<v3u32*>(p) = w;
}

// A tile without bin entries: every pixel is background (sky, id -1, depth
// +inf, normal 0, point NaN) and every in-tile keypoint is visible (its W is
// compared with +inf, as in the general path).  No z-buffer, table or barrier.
__device__ __forceinline__ void empty_tile(const SceneDev& s, const BatchDev& b, uint32_t f, uint32_t tile, int ox,
                                           int oy) {
  const int tid = threadIdx.x;
  if (b.n_kp && ((b.kp_tiles[(size_t)f * b.tile_words + (tile >> 5)] >> (tile & 31u)) & 1u)) {
    for (uint32_t k = tid; k < b.n_kp; k += kRB) {
      const size_t o = (size_t)f * b.n_kp + k;
      const uint32_t pp = b.kp_pix[o];
      const int px = (int)(pp & 0xFFFFu) - ox, py = (int)(pp >> 16) - oy;
      if (pp == 0xFFFFFFFFu || px < 0 || px >= kTileW || py < 0 || py >= kTileH) continue;
      b.kp_vis[o] = (b.kp_w[o] <= INFINITY) ? 2 : 1;
    }
  }
  const int ly = tid / (kTileW / 4), lx0 = (tid % (kTileW / 4)) * 4;
  const int py = oy + ly, px0 = ox + lx0;
  if (py >= (int)s.H) return;
  const size_t o = (size_t)f * s.W * s.H + (size_t)py * s.W + px0;
  const uint32_t sky = b.lights[b.fset[f]].sky & 0xFFFFFFu;
  const float nan = __builtin_nanf("");
  if (px0 + 3 < (int)s.W && ((o + b.px_align) & 3u) == 0) {
    if (b.inst) out_ids(b.inst + o, make_int4(-1, -1, -1, -1));
    if (b.rgb) out_rgb4(b.rgb + o * 3, sky, sky, sky, sky);
    if (b.depth) out_f4(b.depth + o, INFINITY, INFINITY, INFINITY, INFINITY);
    if (b.normals) {
      for (int w = 0; w < 3; ++w) out_u2(b.normals + o * 3 + 4 * w, 0u, 0u);
    }
    if (b.points) {
      for (int w = 0; w < 3; ++w) out_f4(b.points + o * 3 + 4 * w, nan, nan, nan, nan);
    }
  } else {
    for (int k = 0; k < 4 && px0 + k < (int)s.W; ++k) {
      if (b.inst) b.inst[o + k] = -1;
      if (b.rgb) {
        b.rgb[(o + k) * 3 + 0] = (uint8_t)(sky & 255u);
        b.rgb[(o + k) * 3 + 1] = (uint8_t)((sky >> 8) & 255u);
        b.rgb[(o + k) * 3 + 2] = (uint8_t)((sky >> 16) & 255u);
      }
      if (b.depth) b.depth[o + k] = INFINITY;
      if (b.normals) b.normals[(o + k) * 3 + 0] = b.normals[(o + k) * 3 + 1] = b.normals[(o + k) * 3 + 2] = 0;
      if (b.points) b.points[(o + k) * 3 + 0] = b.points[(o + k) * 3 + 1] = b.points[(o + k) * 3 + 2] = nan;
    }
  }
}

// kCov: also the per-label coverage for occlusion (b.covered); a separate
// instantiation launched only when the caller asks for it.  Its coverage table
// (4.1 KiB) is paid for with smaller batches (CSG_COV_STAGE records), so it
// keeps 7 workgroups per CU.
template <bool kCov>
__global__ __launch_bounds__(kRasterBlock) CSG_RASTER_ATTR void k_raster(SceneDev s, BatchDev b) {
  __shared__ unsigned long long zb[kTilePix];        // (depth,uid) keys: 8 KiB at 32 x 32
  constexpr int NS = kStageOf<kCov>;
  __shared__ union Lds {
    RasterSide<kCov> ra;                             // raster loop
    ResolveLds q;                                    // resolve
  } L;
  const int tid = threadIdx.x;
  uint32_t tile;
  if (!swizzled_tile(blockIdx.x, s.tiles_x, s.tiles_y, tile)) return;
  const uint32_t f = blockIdx.y;
  const int ox = (int)(tile % s.tiles_x) * kTileW, oy = (int)(tile / s.tiles_x) * kTileH;
  const uint32_t* toff = b.tile_off + (size_t)f * (s.n_tiles + 1);
  const Slab sb = b.slab[f];
  const uint32_t beg = min(toff[tile], sb.bin_cap);
  const uint32_t end = (DBG(b.dbg) & 2u) ? beg : min(toff[tile + 1], sb.bin_cap);
  if (beg == end && !(DBG(b.dbg) & 2u)) {   // nothing binned here: background only
    empty_tile(s, b, f, tile, ox, oy);
    return;
  }
  const uint32_t* bins = b.bins + sb.bin_base;
  // the first batch's record ids, loaded before the z-buffer initialisation (CSG_PREFETCH_BIN)
  const uint32_t rfirst = (CSG_PREFETCH_BIN && tid < NS && beg + (uint32_t)tid < end) ? bins[beg + tid] : 0xFFFFFFFFu;
  for (int p = tid; p < kTilePix; p += kRB) zb[p] = kEmptyKey;
  CovLds* covp = nullptr;
  int32_t* rlabel = nullptr;
  if constexpr (kCov) {
    covp = &L.ra.cov;
    rlabel = L.ra.rlabel;
    CovLds& covl = *covp;
    for (int p = tid; p < kCovSlots * (kTilePix / 32); p += kRB) (&covl.mask[0][0])[p] = 0u;
    if (tid < kCovSlots) covl.keys[tid] = kNoAlpha;
    if (tid == 0) covl.ovf = 0u;
  }
  const Rec* recs = b.recs + sb.rec_base;
  RasterCtx c{s.aquad, s.acls, zb, ox, oy, s.inv_near, s.inv_far, b.dbg, b.overflow, covp, rlabel,
              kCov ? b.covered + (size_t)f * b.n_labels : nullptr};
  __syncthreads();
  raster_block<kCov, NS>(c, s, b, L.ra.r, beg, end, bins, recs, sb.rec_cap, rfirst);
  __syncthreads();
  if constexpr (kCov) {
    // per slot: popcount of its kTilePix / 32 mask words, kTPS threads per
    // slot (4 words each, consecutive lanes of one wave); the table is
    // read-only from here on
    const CovLds& covl = *covp;
    constexpr int kTPS = kRB / kCovSlots;
    static_assert(kTPS * 4 * 32 == kTilePix && kTPS <= 64, "4 words per thread, a slot's threads in one wave");
    const uint32_t sl = (uint32_t)tid / kTPS, w0 = ((uint32_t)tid % kTPS) * 4u;
    uint32_t n = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) n += (uint32_t)__popc(covl.mask[sl][w0 + w]);
#pragma unroll
    for (int o = 1; o < kTPS; o <<= 1) n += (uint32_t)__shfl_xor((int)n, o, 64);
    const uint32_t lab = covl.keys[sl];
    if ((tid % kTPS) == 0 && lab != kNoAlpha) {
      if (covl.ovf) atomicOr(&c.gcov[lab], kCovUnknown);
      else atomicAdd(&c.gcov[lab], n);
    }
    __syncthreads();   // the resolve reuses the table's LDS
  }

  if (DBG(b.dbg) & 1u) {   // ablation: keep the raster loop alive, skip the resolve
    if (tid == 0 && zb[0] == 0ull && b.inst) b.inst[0] = 0;
    return;
  }
  // keypoint visibility against the finished z-buffer: W <= depth -> 2, else 1
  // (depth = 1/invW of the winning key, the value the resolve writes)
  if (b.n_kp && ((b.kp_tiles[(size_t)f * b.tile_words + (tile >> 5)] >> (tile & 31u)) & 1u)) {
    for (uint32_t k = tid; k < b.n_kp; k += kRB) {
      const size_t o = (size_t)f * b.n_kp + k;
      const uint32_t pp = b.kp_pix[o];
      const int px = (int)(pp & 0xFFFFu) - ox, py = (int)(pp >> 16) - oy;
      if (pp == 0xFFFFFFFFu || px < 0 || px >= kTileW || py < 0 || py >= kTileH) continue;
      const unsigned long long key = zb[zb_index(px, py)];
      const float d = key == kEmptyKey ? INFINITY : rcp_ieee(__uint_as_float(0xFFFFFFFFu - (uint32_t)(key >> 32)));
      b.kp_vis[o] = (b.kp_w[o] <= d) ? 2 : 1;
    }
    // The resolve below overwrites background z-buffer words (with the sky
    // word) before its first barrier: every keypoint must have read its key
    // first.  (Without this barrier a keypoint over the sky could read the sky
    // word, whose depth field is 0: harmless with the IEEE 1/0 = +inf, a NaN
    // with the Newton reciprocal, found by the bench's own verification.)
    // The branch is uniform over the block (frame and tile).
    __syncthreads();
  }
  // Label statistics (pixel count + tight box per label) only when the caller
  // asked for them (csg_outputs.inst_stats): otherwise no LDS table, no runs.
  const bool want_stats = b.stats != nullptr;
  const uint32_t nl = want_stats ? min(b.n_labels, (uint32_t)kMaxLdsLabels) : 0u;
  uint32_t (*lstat)[kMaxLdsLabels] = L.q.lstat;   // [0] count, [1] row mask, [2..] column masks
  for (uint32_t l = tid; l < nl; l += kRB) {
#pragma unroll
    for (int w = 0; w < 2 + kColWords; ++w) lstat[w][l] = 0;
  }
  // ---- resolve: 4 consecutive pixels per thread, one tile row per 8 threads.
  // Rounds: the tile's distinct winning triangles go into the shade table
  // (up to kShadeSlots per round), each is set up once by one thread, then
  // every pixel showing it is shaded from the table.  Pixels whose triangle
  // found no slot wait for the next round (normally there is one round).
  // A shaded pixel's z-buffer word is dead, so it takes the pixel's result
  // (rgb | id << 32) until the vector stores at the end: between phases a
  // thread keeps only bit masks and slot numbers in registers.
  const int ly = tid / (kTileW / 4), lx0 = (tid % (kTileW / 4)) * 4;
  const int py = oy + ly;
  const bool row_ok = py < (int)s.H;
  const int px0 = ox + lx0;
  // this thread's 4 pixels: the aligned 4-word group at zb_index(lx0, ly) & ~3,
  // pixel k in word k ^ (ly & 3) of it (zpix)
  unsigned long long* zrow = &zb[zb_index(lx0, ly) & ~3];
  const int zsw = CSG_ZB_SWIZZLE ? (ly & 3) : 0;
  auto zpix = [&](int k) -> unsigned long long& { return zrow[k ^ zsw]; };
  uint32_t pend = 0;                 // bit k: pixel k still to shade
  uint32_t inmask = 0;               // bit k: pixel k lies inside the frame
  // The depth visualisation's range (b.drange), from the winning keys: the
  // written depth is 1/invW (IEEE, monotone), so the tile's smallest depth is
  // 1/(largest invW), i.e. comes from the smallest key.  Reduced per wave here;
  // thread 0 combines the waves after the first round's barrier.
  __shared__ uint32_t drw[2][kRB / 64];
  {
    const uint32_t sky = b.lights[b.fset[f]].sky & 0xFFFFFFu;
    const unsigned long long bgword = (unsigned long long)sky | (0xFFFFFFFFull << 32);   // id -1
    uint32_t kmn = 0xFFFFFFFFu, kmx = 0u;   // key high words (0xFFFFFFFF - bits(invW))
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const bool in = row_ok && px0 + k < (int)s.W;
      inmask |= in ? 1u << k : 0u;
      const unsigned long long key = zpix(k);
      if (in && key != kEmptyKey) {
        pend |= 1u << k;
        kmn = min(kmn, (uint32_t)(key >> 32));
        kmx = max(kmx, (uint32_t)(key >> 32));
      } else {
        zpix(k) = bgword;            // background (or outside the frame)
      }
    }
    if (b.drange) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        kmn = min(kmn, (uint32_t)__shfl_xor((int)kmn, o, 64));
        kmx = max(kmx, (uint32_t)__shfl_xor((int)kmx, o, 64));
      }
      if ((tid & 63) == 0) { drw[0][tid >> 6] = kmn; drw[1][tid >> 6] = kmx; }
    }
  }
  const size_t npx = (size_t)s.W * s.H;
  const size_t o = (size_t)f * npx + (size_t)py * s.W + px0;
  // background pixels inside the frame (a pixel past the right edge would
  // address the next row's first pixels: per-pixel depth / normal / point
  // stores must not see it)
  const uint32_t bgmask = inmask & ~pend;
  const bool need_depth = b.depth || b.points;
  // One round; returns whether any pixel of the tile is left.  The first
  // round is peeled off (called outside the loop) so the compiler does not
  // hoist per-pixel invariants across the setup phase, where they would spill.
  auto round = [&](const bool first) __attribute__((always_inline)) -> bool {
    if ((uint32_t)tid < kShadeSlots) L.q.keys[tid] = kNoAlpha;
    __syncthreads();
    // every thread has read the previous round's flag (it reached this
    // barrier) and none sets it before the next barrier
    if (tid == 0) L.q.more = 0;
    if (first && b.drange && tid == 0) {   // the tile's depth range (see drw)
      uint32_t kmn = drw[0][0], kmx = drw[1][0];
#pragma unroll
      for (int w = 1; w < kRB / 64; ++w) { kmn = min(kmn, drw[0][w]); kmx = max(kmx, drw[1][w]); }
      if (kmn <= kmx) {   // some pixel has a surface: depths 1/invW, valid (finite, > 0) by the depth range test
        const float dmin = rcp_ieee(__uint_as_float(0xFFFFFFFFu - kmn));
        const float dmax = rcp_ieee(__uint_as_float(0xFFFFFFFFu - kmx));
        // skip the atomic when the frame's range already holds it (most tiles)
        if (__float_as_uint(dmin) < b.drange[f]) atomicMin(&b.drange[f], __float_as_uint(dmin));
        if (__float_as_uint(dmax) > b.drange[b.drange_F + f]) atomicMax(&b.drange[b.drange_F + f], __float_as_uint(dmax));
      }
    }
    uint32_t slots = 0xFFFFFFFFu;    // 8 bits per pixel (0xFF: none this round)
    {
      uint32_t prev_uid = 0xFFFFFFFFu, prev_slot = 0xFFu;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if ((pend >> k) & 1u) {
          const uint32_t uid = (uint32_t)zpix(k);
          uint32_t sl;
          if (uid == prev_uid) sl = prev_slot;
          else {
            const int r = shade_slot(L.q.keys, uid);
            sl = r < 0 ? 0xFFu : (uint32_t)r;
          }
          prev_uid = uid;
          prev_slot = sl;
          slots = (slots & ~(0xFFu << (8 * k))) | (sl << (8 * k));
        } else {
          prev_uid = 0xFFFFFFFFu;
        }
      }
    }
    __syncthreads();
    {  // one thread per occupied slot: set the triangle up once for the whole tile
      const uint32_t u = (uint32_t)tid < kShadeSlots ? L.q.keys[tid] : kNoAlpha;
      if (u != kNoAlpha) {
        ShadeEntry& e = L.q.tab[tid];
        if (DBG(b.dbg) & 8192u) {   // ablation only: no triangle setup (garbage shading)
          e = ShadeEntry{};
          e.P[2] = 1.0f; e.tex = -1; e.label = 0;
        } else {
          shade_setup(s, b, f, u, e);
        }
      }
    }
    __syncthreads();
    if (row_ok) {
      // pixel coordinates laundered through an empty asm: everything derived
      // from them is computed here, not hoisted across the setup phase above
      // (it would be live there and spill)
      int qx0 = px0, qy = py;
      asm volatile("" : "+v"(qx0), "+v"(qy));
      const size_t qo = (size_t)f * npx + (size_t)qy * s.W + qx0;
      int32_t run = -1;              // label stats, one set of LDS atomics per run of equal labels
      uint32_t cnt = 0, xmin = 0, xmax = 0;
      auto flush_run = [&]() {
        if (DBG(b.dbg) & 16384u) return;   // ablation only: no label stats
        if (run >= 0 && (uint32_t)run < nl) {
          // the box as bit masks of the tile's columns and rows: 3 atomics per
          // run instead of 5 (min/max are the lowest and highest bits)
          // (a run lies inside one thread's 4 pixels: one column word)
          const uint32_t col = xmin - (uint32_t)ox;
          atomicAdd(&lstat[0][run], cnt);
          atomicOr(&lstat[2 + (kColWords > 1 ? col >> 5 : 0u)][run], (0xFu >> (3u - (xmax - xmin))) << (col & 31u));
          atomicOr(&lstat[1][run], 1u << ((uint32_t)qy - (uint32_t)oy));
        } else if (run >= 0 && b.stats && (uint32_t)run < b.n_labels) {   // beyond the LDS table
          uint32_t* st = b.stats + ((size_t)f * b.n_labels + (uint32_t)run) * 5;
          atomicAdd(&st[0], cnt);
          atomicMin(&st[1], xmin);
          atomicMin(&st[2], (uint32_t)qy);
          atomicMax(&st[3], xmax);
          atomicMax(&st[4], (uint32_t)qy);
        }
      };
      // The optional per-pixel outputs (depth, normals, points) of a group
      // whose 4 pixels all lie in the frame and are all finished in this round
      // go out after the loop as one 16-B depth, three 8-B normal and three
      // 16-B point stores (lane-contiguous); otherwise, and with CSG_VEC_OUT 0,
      // each pixel stores its own (4-B, 2-B and 4-B stores at 16-, 6- and 12-B
      // pixel strides: at 4K those narrow stores were 30% of k_raster).
      // (o % 4 == 0 keeps the group's outputs 16-B aligned, as in empty_tile.)
      bool vec = false;
      if (CSG_VEC_OUT && (b.depth || b.normals || b.points) && inmask == 0xFu && ((qo + b.px_align) & 3u) == 0) {
        uint32_t done = first ? bgmask : 0u;
#pragma unroll
        for (int k = 0; k < 4; ++k) done |= ((slots >> (8 * k)) & 0xFFu) != 0xFFu ? 1u << k : 0u;
        vec = done == 0xFu;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int px = qx0 + k;
        const uint32_t sl = (slots >> (8 * k)) & 0xFFu;
        // background pixels are written in the first round; the optional
        // outputs of a pixel not in a vector group are stored per pixel
        const bool bg = first && ((bgmask >> k) & 1u);
        if (sl == 0xFFu && !bg) continue;
        float dep = INFINITY;
        uint32_t n01 = 0, n2 = 0;
        if (!bg) {
          const ShadeEntry& e = L.q.tab[sl];
          uint32_t rgb;
          int32_t id;
          // (a vector group's depths are evaluated again after the loop)
          shade_pixel(s, e, px, qy, need_depth && !(CSG_VEC_DEP_ONCE && vec), rgb, id, dep);
          n01 = e.n01;
          n2 = e.n2;
          zpix(k) = (unsigned long long)rgb | ((unsigned long long)(uint32_t)id << 32);
          pend &= ~(1u << k);
          if (want_stats) {
            if (id != run) {
              flush_run();
              run = id;
              cnt = 0;
              xmin = (uint32_t)px;
            }
            ++cnt;
            xmax = (uint32_t)px;
          }
        }
        if (vec) continue;
        if (b.depth) b.depth[qo + k] = dep;
        if (b.normals) {
          uint16_t* d = b.normals + (qo + k) * 3;
          d[0] = (uint16_t)(n01 & 0xFFFFu);
          d[1] = (uint16_t)(n01 >> 16);
          d[2] = (uint16_t)n2;
        }
        if (b.points) {
          float pt[3];
          if (bg) pt[0] = pt[1] = pt[2] = __builtin_nanf("");
          else unproject(b.cam + (size_t)f * kCamFloats, px, qy, dep, pt);
          float* d = b.points + (qo + k) * 3;
          d[0] = pt[0];
          d[1] = pt[1];
          d[2] = pt[2];
        }
      }
      flush_run();
      if (vec) {   // background pixels (first round): depth +inf, normal 0, point NaN
        // the depths again, from the table (as shade_pixel: the same bits), so
        // that none is live across the shading loop
        const uint32_t bgv = first ? bgmask : 0u;
        float dv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const ShadeEntry& e = L.q.tab[(bgv >> k) & 1u ? 0u : (slots >> (8 * k)) & 0xFFu];
          const float fx = (float)(qx0 + k) + 0.5f, fy = (float)qy + 0.5f;
          dv[k] = ((bgv >> k) & 1u) || !need_depth ? INFINITY : rcp_ieee(plane_at(e.P[0], e.P[1], e.P[2], fx, fy));
        }
        if (b.depth) out_f4(b.depth + qo, dv[0], dv[1], dv[2], dv[3]);
        if (b.normals) {   // 12 halves x0 y0 z0 x1 ... z3 as 6 words
          uint32_t n01[4], n2[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const bool bg = (bgv >> k) & 1u;
            const ShadeEntry& e = L.q.tab[bg ? 0u : (slots >> (8 * k)) & 0xFFu];
            n01[k] = bg ? 0u : e.n01;
            n2[k] = bg ? 0u : e.n2;
          }
          uint16_t* d = b.normals + qo * 3;
          out_u2(d, n01[0], n2[0] | (n01[1] << 16));
          out_u2(d + 4, (n01[1] >> 16) | (n2[1] << 16), n01[2]);
          out_u2(d + 8, n2[2] | (n01[3] << 16), (n01[3] >> 16) | (n2[3] << 16));
        }
        if (b.points) {
          float pt[12];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            if ((bgv >> k) & 1u) pt[3 * k] = pt[3 * k + 1] = pt[3 * k + 2] = __builtin_nanf("");
            else unproject(b.cam + (size_t)f * kCamFloats, qx0 + k, qy, dv[k], pt + 3 * k);
          }
          float* d = b.points + qo * 3;
          out_f4(d, pt[0], pt[1], pt[2], pt[3]);
          out_f4(d + 4, pt[4], pt[5], pt[6], pt[7]);
          out_f4(d + 8, pt[8], pt[9], pt[10], pt[11]);
        }
      }
    }
    if (pend) L.q.more = 1;          // (__syncthreads_or measured 16% slower here)
    __syncthreads();
    return L.q.more != 0;
  };
  if (round(true)) {
#pragma clang loop unroll(disable)
    while (round(false)) {
    }
  }
  if (row_ok) {
    uint32_t rgb[4];
    int32_t ids[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const unsigned long long w = zpix(k);
      rgb[k] = (uint32_t)w;
      ids[k] = (int32_t)(w >> 32);
    }
    if (px0 + 3 < (int)s.W && ((o + b.px_align) & 3u) == 0) {
      if (b.inst) out_ids(b.inst + o, make_int4(ids[0], ids[1], ids[2], ids[3]));
      if (b.rgb) out_rgb4(b.rgb + o * 3, rgb[0], rgb[1], rgb[2], rgb[3]);
    } else {
      for (int k = 0; k < 4 && px0 + k < (int)s.W; ++k) {
        if (b.inst) b.inst[o + k] = ids[k];
        if (b.rgb) {
          b.rgb[(o + k) * 3 + 0] = (uint8_t)(rgb[k] & 255u);
          b.rgb[(o + k) * 3 + 1] = (uint8_t)((rgb[k] >> 8) & 255u);
          b.rgb[(o + k) * 3 + 2] = (uint8_t)((rgb[k] >> 16) & 255u);
        }
      }
    }
  }
  if (b.stats) {
    __syncthreads();
    uint32_t* st = b.stats + (size_t)f * b.n_labels * 5;
    for (uint32_t l = tid; l < nl; l += kRB) {
      const uint32_t cnt = lstat[0][l];
      if (cnt) {
        const uint32_t rm = lstat[1][l];
        uint32_t cm = lstat[2][l], cm_hi = cm, lo_w = 0, hi_w = 0;   // column words: first / last non-empty
#pragma unroll
        for (int w = 1; w < kColWords; ++w) {
          const uint32_t m = lstat[2 + w][l];
          if (!cm && m) { cm = m; lo_w = (uint32_t)w; }
          if (m) { cm_hi = m; hi_w = (uint32_t)w; }
        }
        if (!cm_hi) cm_hi = cm;
        atomicAdd(&st[l * 5 + 0], cnt);
        atomicMin(&st[l * 5 + 1], (uint32_t)ox + 32u * lo_w + (uint32_t)(__ffs(cm) - 1));
        atomicMin(&st[l * 5 + 2], (uint32_t)oy + (uint32_t)(__ffs(rm) - 1));
        atomicMax(&st[l * 5 + 3], (uint32_t)ox + 32u * hi_w + 31u - (uint32_t)__clz(cm_hi));
        atomicMax(&st[l * 5 + 4], (uint32_t)oy + 31u - (uint32_t)__clz(rm));
      }
    }
  }
}

__global__ void k_init_stats(uint32_t* st, uint32_t n) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) {
    const uint32_t c = k % 5;
    st[k] = (c == 1 || c == 2) ? 0xFFFFFFFFu : 0u;
  }
}

// ---------------------------------------------------------------------------
// k_keypoints: projection of the frame's keypoints (before k_raster).  The
// depth test that turns "in view" (1) into "visible" (2) runs inside k_raster
// against the finished z-buffer, so the depth image need not exist in HBM.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void project_one(const float* pv, const float* p, float Wf, float Hf, float nearc,
                                            float& u, float& v, int& vis, int& px, int& py) {
  const float X = dot4(pv + 0, p[0], p[1], p[2]);
  const float Y = dot4(pv + 4, p[0], p[1], p[2]);
  const float Wc = dot4(pv + 8, p[0], p[1], p[2]);
  px = py = -1;
  if (!(Wc >= nearc)) {
    u = -1.0f; v = -1.0f; vis = 0;
    return;
  }
  u = X / Wc;
  v = Y / Wc;
  if (!(u >= 0.0f && u < Wf && v >= 0.0f && v < Hf)) { vis = 0; return; }
  px = (int)u;
  py = (int)v;
  vis = 1;
}

__global__ __launch_bounds__(256) void k_keypoints(SceneDev s, BatchDev b) {
  const uint32_t f = blockIdx.y;
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= b.n_kp) return;
  const float* pv = b.pv + (size_t)f * 12;
  const size_t o = (size_t)f * b.n_kp + k;
  const uint32_t kset = b.frames[f].xform_set;
  if (kset >= b.n_kp_sets) {   // device frame without keypoints for its set: nothing projected
    b.kp_uv[o * 2 + 0] = -1.0f;
    b.kp_uv[o * 2 + 1] = -1.0f;
    b.kp_vis[o] = 0;
    b.kp_pix[o] = 0xFFFFFFFFu;
    b.kp_w[o] = INFINITY;
    if (k == 0) atomicOr(b.overflow, kOvBadKpSet);
    return;
  }
  const float* p = b.kp + ((size_t)kset * b.n_kp + k) * 3;
  float u, v;
  int vis, px, py;
  project_one(pv, p, (float)s.W, (float)s.H, s.near_clip, u, v, vis, px, py);
  b.kp_uv[o * 2 + 0] = u;
  b.kp_uv[o * 2 + 1] = v;
  b.kp_vis[o] = vis;
  b.kp_pix[o] = vis ? ((uint32_t)px | ((uint32_t)py << 16)) : 0xFFFFFFFFu;
  b.kp_w[o] = dot4(pv + 8, p[0], p[1], p[2]);
  if (vis) {
    const uint32_t t = (uint32_t)(py / kTileH) * s.tiles_x + (uint32_t)(px / kTileW);
    atomicOr(&b.kp_tiles[(size_t)f * b.tile_words + (t >> 5)], 1u << (t & 31u));
  }
}

// ---------------------------------------------------------------------------
// k_inst_bounds: world-space AABB of every instance's vertices under one
// transform set (3D bbox annotator, GDP:1780-1790).  One block per chunk;
// wave min/max, then order-preserving uint atomics (decoded on the host).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t ordered_bits(float x) {
  const uint32_t u = __float_as_uint(x);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ __launch_bounds__(256) void k_inst_bounds(SceneDev s, const Chunk* __restrict__ chunks,
                                                     const float* __restrict__ models, uint32_t* __restrict__ out) {
  const Chunk& ch = chunks[blockIdx.x];
  const int tid = threadIdx.x;
  const uint32_t i = ch.inst;
  float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  if ((uint32_t)tid < ch.count) {
    const float* M = models + (size_t)i * 16;
    float m[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) m[k] = M[k];
    const float* tp = s.tri_pos + (size_t)(ch.soup + tid) * 9;
#pragma unroll
    for (int v = 0; v < 3; ++v) {
      const float x = tp[3 * v], y = tp[3 * v + 1], z = tp[3 * v + 2];
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        const float w = dot4(m + 4 * a, x, y, z);
        lo[a] = fminf(lo[a], w);
        hi[a] = fmaxf(hi[a], w);
      }
    }
  }
#pragma unroll
  for (int a = 0; a < 3; ++a) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
      lo[a] = fminf(lo[a], __shfl_xor(lo[a], d, 64));
      hi[a] = fmaxf(hi[a], __shfl_xor(hi[a], d, 64));
    }
  }
  if ((tid & 63) == 0 && (uint32_t)tid < ch.count) {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      atomicMin(&out[i * 6 + a], ordered_bits(lo[a]));
      atomicMax(&out[i * 6 + 3 + a], ordered_bits(hi[a]));
    }
  }
}

__global__ void k_project(const float* pts, uint32_t n, const float* pv, float Wf, float Hf, float nearc, float* uv,
                          int32_t* vis) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  float u, v;
  int vs, px, py;
  project_one(pv, pts + (size_t)k * 3, Wf, Hf, nearc, u, v, vs, px, py);
  uv[2 * k] = u;
  uv[2 * k + 1] = v;
  vis[k] = vs;
}

// ---------------------------------------------------------------------------
// Depth visualisation (GDP:1690-1709): the reference normalises the valid
// depth (finite, > 0) of each frame by its min / max and maps it through
// OpenCV's JET colour map.  The per-frame min / max come from k_raster's
// resolve (b.drange: the winning keys' depths, reduced per tile); this pass
// streams the depth image once for the colour lookup (HBM-bound).
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool depth_valid(float d) { return d > 0.0f && d < INFINITY; }

// Index of one depth value (GDP:1698-1700, NumPy 1.x promotion as Isaac Sim
// runs it): (depth_max - depth_min) is a float32 scalar, + 1e-6 promotes it to
// float64, and dividing the float32 array by that scalar casts it back to
// float32; then ((d - min) / den) * 255 in float32 and astype(uint8) truncates.
__device__ __forceinline__ uint32_t depth_index(float v, float mn, float den) {
  if (!depth_valid(v)) return 0u;
  const int q = (int)(((v - mn) / den) * 255.0f);
  return (uint32_t)min(max(q, 0), 255);
}

template <bool kVec>
__global__ __launch_bounds__(256) void k_depth_vis(const float* __restrict__ depth, uint32_t npx, uint32_t F,
                                                   const uint32_t* __restrict__ range, const uint32_t* __restrict__ lut,
                                                   uint8_t* __restrict__ vis, float* __restrict__ range_out) {
  __shared__ uint32_t tab[256];
  const uint32_t f = blockIdx.y;
  tab[threadIdx.x] = lut[threadIdx.x];
  const uint32_t mnb = range[f], mxb = range[F + f];
  const bool any = mnb != 0xFFFFFFFFu;          // no valid depth: the reference writes a black image
  const float mn = __uint_as_float(mnb), mx = __uint_as_float(mxb);
  const float den = (float)((double)(mx - mn) + 1e-6);
  if (range_out && blockIdx.x == 0 && threadIdx.x == 0) {
    range_out[2 * f] = any ? mn : __builtin_nanf("");
    range_out[2 * f + 1] = any ? mx : __builtin_nanf("");
  }
  __syncthreads();
  if (!vis) return;       // range only
  const size_t base = (size_t)f * npx;
  if constexpr (kVec) {   // 4 pixels per thread: one float4 in, three dwords out
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= npx / 4u) return;
    const float4 v = reinterpret_cast<const float4*>(depth + base)[q];
    uint32_t c[4] = {0u, 0u, 0u, 0u};
    if (any) {
      c[0] = tab[depth_index(v.x, mn, den)];
      c[1] = tab[depth_index(v.y, mn, den)];
      c[2] = tab[depth_index(v.z, mn, den)];
      c[3] = tab[depth_index(v.w, mn, den)];
    }
    uint32_t* o = reinterpret_cast<uint32_t*>(vis + (base + 4u * (size_t)q) * 3);
    o[0] = c[0] | (c[1] << 24);
    o[1] = (c[1] >> 8) | (c[2] << 16);
    o[2] = (c[2] >> 16) | (c[3] << 8);
  } else {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= npx) return;
    const uint32_t c = any ? tab[depth_index(depth[base + i], mn, den)] : 0u;
    uint8_t* o = vis + (base + i) * 3;
    o[0] = (uint8_t)(c & 255u);
    o[1] = (uint8_t)((c >> 8) & 255u);
    o[2] = (uint8_t)((c >> 16) & 255u);
  }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
void launch_clip(const SceneDev& s, const BatchDev& b, uint32_t F, hipStream_t st) {
  dim3 g((s.n_inst + 255) / 256, F);
  hipLaunchKernelGGL(k_clip, g, dim3(256), 0, st, s, b);
}

void launch_setup(const SceneDev& s, const BatchDev& b, const Chunk* chunks, uint32_t n_chunks, uint32_t F,
                  hipStream_t st) {
  const uint32_t gy = n_chunks < 65535u ? n_chunks : 65535u;   // grid y limit
  dim3 g(F, gy, (n_chunks + gy - 1) / gy);
  hipLaunchKernelGGL(k_setup, g, dim3(kBlock), 0, st, s, b, chunks, n_chunks);
}

void launch_count(const SceneDev& s, const BatchDev& b, uint32_t F, uint32_t blocks, hipStream_t st) {
  const uint32_t band = s.n_tiles < kBinBand ? s.n_tiles : kBinBand;
  const size_t lds = (((band + 3u) & ~3u) + 2 * kBinRound + 12) * sizeof(uint32_t);
  // (one band: the kernels without the per-entry band test)
  if (s.n_tiles > kBinBand) hipLaunchKernelGGL(k_count<true>, dim3(blocks, F), dim3(kBlock), lds, st, s, b);
  else hipLaunchKernelGGL(k_count<false>, dim3(blocks, F), dim3(kBlock), lds, st, s, b);
}

void launch_plan(const FrameDev* frames, uint32_t F, uint32_t def_rec, uint32_t def_bin, uint64_t rec_pool,
                 uint64_t bin_pool, int use_hints, Slab* slab, uint64_t* need, hipStream_t st) {
  hipLaunchKernelGGL(k_plan, dim3(1), dim3(64), 0, st, frames, F, def_rec, def_bin, rec_pool, bin_pool, use_hints,
                     slab, need);
}

void launch_scan(const SceneDev& s, const BatchDev& b, uint32_t F, hipStream_t st) {
  hipLaunchKernelGGL(k_scan, dim3(F), dim3(kBlock), 0, st, s, b);
}

void launch_bin(const SceneDev& s, const BatchDev& b, uint32_t F, uint32_t blocks, hipStream_t st) {
  dim3 g(blocks, F);
  const uint32_t band = s.n_tiles < kBinBand ? s.n_tiles : kBinBand;
  if (s.n_tiles > kBinBand) hipLaunchKernelGGL(k_bin<true>, g, dim3(kBlock), band * sizeof(uint32_t), st, s, b);
  else hipLaunchKernelGGL(k_bin<false>, g, dim3(kBlock), band * sizeof(uint32_t), st, s, b);
}

void launch_colscan(const SceneDev& s, const BatchDev& b, uint32_t F, hipStream_t st) {
  hipLaunchKernelGGL(k_colscan, dim3((s.n_tiles + kBlock - 1) / kBlock, F), dim3(kBlock), 0, st, s, b);
}

void launch_raster(const SceneDev& s, const BatchDev& b, uint32_t F, hipStream_t st) {
  const uint32_t squares = ((s.tiles_x + kSqX - 1) / kSqX) * ((s.tiles_y + kSqY - 1) / kSqY);
  dim3 g(8 * kSqN * ((squares + 7) / 8), F);
  if (b.covered) hipLaunchKernelGGL(k_raster<true>, g, dim3(kRasterBlock), 0, st, s, b);
  else hipLaunchKernelGGL(k_raster<false>, g, dim3(kRasterBlock), 0, st, s, b);
}

void launch_init_stats(const BatchDev& b, uint32_t F, hipStream_t st) {
  const uint32_t n = F * b.n_labels * 5;
  if (!n || !b.stats) return;
  hipLaunchKernelGGL(k_init_stats, dim3((n + 255) / 256), dim3(256), 0, st, b.stats, n);
}

void launch_keypoints(const SceneDev& s, const BatchDev& b, uint32_t F, hipStream_t st) {
  if (!b.n_kp) return;
  dim3 g((b.n_kp + 255) / 256, F);
  hipLaunchKernelGGL(k_keypoints, g, dim3(256), 0, st, s, b);
}

void launch_inst_bounds(const SceneDev& s, const Chunk* chunks, uint32_t n_chunks, const float* models,
                        uint32_t* out, hipStream_t st) {
  hipLaunchKernelGGL(k_inst_bounds, dim3(n_chunks), dim3(kBlock), 0, st, s, chunks, models, out);
}

void launch_project(const float* pts, uint32_t n, const float* pv12, float W, float H, float near_clip, float* uv,
                    int32_t* vis, hipStream_t st) {
  hipLaunchKernelGGL(k_project, dim3((n + 255) / 256), dim3(256), 0, st, pts, n, pv12, W, H, near_clip, uv, vis);
}

void launch_depth_vis(const float* depth, uint32_t npx, uint32_t F, const uint32_t* range, const uint32_t* lut,
                      uint8_t* vis, float* range_out, hipStream_t st) {
  const bool vec = (npx % 4u) == 0 && ((uintptr_t)depth & 15u) == 0 && ((uintptr_t)vis & 3u) == 0;
  const uint32_t items = vec ? npx / 4u : npx;
  dim3 g(vis ? (items + 255u) / 256u : 1u, F);
  if (vec) hipLaunchKernelGGL(k_depth_vis<true>, g, dim3(256), 0, st, depth, npx, F, range, lut, vis, range_out);
  else hipLaunchKernelGGL(k_depth_vis<false>, g, dim3(256), 0, st, depth, npx, F, range, lut, vis, range_out);
}

// ---------------------------------------------------------------------------
// k_narrow_ids: a launch chain's int32 instance ids (-1 background) as
// (id + 1) in `bytes` = 1 or 2 bytes, the host wire of csg_api.cpp's
// host-output batches (csg_widen.h widens them back).  Ids [lo, hi) of `src`,
// absolute indices (src and dst are the batch buffers, 16-B aligned), 4 per
// thread: one 16-B load and one 4-B / 8-B store; ids outside [lo, hi) of a
// thread's aligned group are left alone.  HBM-bound: 4 B read + 1-2 B written per id.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_narrow_ids(const int32_t* __restrict__ src, size_t lo, size_t hi,
                                                     uint32_t bytes, void* __restrict__ dst) {
  const size_t j = (lo & ~(size_t)3) + ((size_t)blockIdx.x * 256u + threadIdx.x) * 4u;
  if (j >= hi) return;
  if (j >= lo && j + 4 <= hi) {
    const v4i32 v = __builtin_nontemporal_load(reinterpret_cast<const v4i32*>(src + j));
    if (bytes == 1) {
      const uint32_t w = ((uint32_t)(v.x + 1) & 255u) | (((uint32_t)(v.y + 1) & 255u) << 8) |
                         (((uint32_t)(v.z + 1) & 255u) << 16) | ((uint32_t)(v.w + 1) << 24);
      *reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(dst) + j) = w;
    } else {
      const uint2 w = make_uint2(((uint32_t)(v.x + 1) & 0xFFFFu) | ((uint32_t)(v.y + 1) << 16),
                                 ((uint32_t)(v.z + 1) & 0xFFFFu) | ((uint32_t)(v.w + 1) << 16));
      *reinterpret_cast<uint2*>(static_cast<uint16_t*>(dst) + j) = w;
    }
    return;
  }
  for (size_t k = j; k < j + 4 && k < hi; ++k) {
    if (k < lo) continue;
    if (bytes == 1) static_cast<uint8_t*>(dst)[k] = (uint8_t)(src[k] + 1);
    else static_cast<uint16_t*>(dst)[k] = (uint16_t)(src[k] + 1);
  }
}

void launch_narrow_ids(const int32_t* src, size_t lo, size_t hi, uint32_t bytes, void* dst, hipStream_t st) {
  const size_t groups = (hi - (lo & ~(size_t)3) + 3) / 4;
  if (!groups) return;
  hipLaunchKernelGGL(k_narrow_ids, dim3((uint32_t)((groups + 255) / 256)), dim3(256), 0, st, src, lo, hi, bytes, dst);
}

}  // namespace csg
