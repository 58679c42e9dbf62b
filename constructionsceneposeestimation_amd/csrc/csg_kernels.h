// Internal interface between the C-ABI host code (csg_api.cpp) and the
// gfx950 kernels (csg_kernels.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace csg {

// Screen tiles: one k_raster workgroup each, 4 consecutive pixels of a tile
// row per thread in the resolve.  32 x 16 (512 pixels, 128-thread / 2-wave
// workgroups) is the production shape since round 5: against 32 x 32 (256
// threads) k_raster -1.8%, frames/s +0.7% with 16 binning blocks per frame
// (C3, 2,880 frames per step; 64 x 16 +3.7%, 16 x 16 +17% raster;
// profiles/r05/ab/tile_shape.md).  CSG_TILE_W / CSG_TILE_H build the others.
#ifndef CSG_TILE_W
#define CSG_TILE_W 32
#endif
#ifndef CSG_TILE_H
#define CSG_TILE_H 16
#endif
constexpr int kTileW = CSG_TILE_W;           // tile width (pixels)
constexpr int kTileH = CSG_TILE_H;           // tile height (pixels)
constexpr int kTilePix = kTileW * kTileH;
constexpr int kRasterBlock = kTilePix / 4;   // k_raster threads per workgroup
static_assert((kTileW == 16 || kTileW == 32 || kTileW == 64) && (kTileH == 16 || kTileH == 32) &&
                  kRasterBlock >= 64 && kRasterBlock <= 256,
              "tile shapes: width 16/32/64, height 16/32, 64..256 threads");
constexpr int kBlock = 256;
constexpr uint32_t kUidShift = 20;        // spec: uid = (instance << 20) | triangle (tie order); see SceneDev::uid_shift
constexpr uint32_t kMaxInstances = 1u << (32 - kUidShift);
constexpr uint32_t kMaxTrisPerMesh = 1u << kUidShift;
#ifndef CSG_LDS_LABELS   // per-label pixel stats kept in k_raster's LDS (the rest: global atomics)
#define CSG_LDS_LABELS ((CSG_TILE_W) * (CSG_TILE_H) >= 1024 ? 256 : 64)   // C3-C5 have 45 labels
#endif
constexpr int kMaxLdsLabels = CSG_LDS_LABELS;
constexpr int kCovSlots = 32;             // labels per tile in k_raster's coverage table (occlusion)
constexpr uint32_t kCovUnknown = 0x80000000u;   // covered[] flag: a tile held more than kCovSlots labels
constexpr uint32_t kCounterStride = 64;   // u32s between per-frame counters: one 256-B line each
constexpr uint32_t kNoAlpha = 0xFFFFFFFFu;  // Rec::atex of a record without alpha test
constexpr uint32_t kCamFloats = 16;         // per-frame unprojection constants (frame_camera)

struct MeshDesc { uint32_t vbase, tbase, ntris, uvbase, has_uv, material; };   // host-side bookkeeping
// Per instance, everything a kernel needs before touching its triangles (one load).
struct InstDesc { uint32_t tbase, material, has_uv; int32_t label; };
struct MatDesc { uint8_t base[4]; int32_t texture; uint32_t alpha_test, alpha_threshold; };
// One instance's material in one transform set, resolved on the host (texture
// swaps applied, texture descriptor inlined): k_setup and the resolve read it
// with one load that depends only on (set, instance).
struct InstSetDev {
  int32_t tex;        // texture sampled by the resolve (-1: flat albedo; also -1 without uvs)
  uint32_t base;      // albedo multiplier r | g << 8 | b << 16
  uint32_t atex;      // alpha test: texel offset of the texture (kNoAlpha: none)
  uint32_t atex_wh;   // alpha texture width | height << 16
  uint32_t athr;      // alpha threshold
  int32_t label;      // the instance's label
  uint32_t alpha_uv;  // alpha-tested material on a mesh with uvs (the record carries uv planes)
  uint32_t pad;
};
static_assert(sizeof(InstSetDev) == 32, "InstSetDev layout");
struct TexDesc { uint32_t offset, width, height, pad; };
// Lighting of one transform set (randomisation epoch): dome (ambient) and
// distant-light contributions per channel, unit direction toward the sun,
// background colour r | g << 8 | b << 16.
struct LightDev { float ambient[3], sun[3], sun_dir[3]; uint32_t sky; };
struct Chunk {                    // <= 256 triangles of one instance + their object-space AABB
  uint32_t inst, start, count;
  uint32_t soup;                  // soup index of triangle `start` (the mesh's base + start)
  float lo[3], hi[3];
  uint32_t pad2[2];
};
static_assert(sizeof(Chunk) == 48, "Chunk layout");

// One raster (sub-)triangle: fixed-point screen vertices for coverage plus the
// screen-space planes of its ORIGINAL triangle (spec §3.5-6): 1/W and, for
// alpha-tested materials, u/W and v/W.  Field groups of 16 B as k_setup
// writes and k_raster stages them: 0 x0 x1 x2 y0 | 1 y1 y2 p0 p1 |
// 2 uid atex D0 D1 | 3 U0 V0 U1 V1 | 4 U2 V2 D2 atex_wh.  The u and v planes
// are interleaved so that (U_k, V_k) is an aligned register pair after the
// 16-B LDS read: k_raster evaluates both planes with packed FP32
// (v_pk_mul_f32 / v_pk_add_f32), each component in the spec's order.
struct __attribute__((aligned(16))) Rec {
  int32_t x[3], y[3];          // 24: 24.8 fixed point, positive orientation
  uint16_t px0, py0, px1, py1; // 8 : inclusive pixel bbox, clamped to the frame
  uint32_t uid;                // 4
  uint32_t atex;               // 4 : alpha test (kNoAlpha: none): texel offset / 16 | threshold << 24
                               //     (keep iff alpha > threshold; texture offsets are 16-texel aligned)
  float D0, D1;                // 8 : 1/W = (D0*x + D1*y) + D2 at pixel centre (x, y)
  float UV[3][2];              // 24: (u/W, v/W) plane coefficient pairs (alpha-tested materials; zeros otherwise)
  float D2;                    // 4
  uint32_t atex_wh;            // 4 : alpha texture width | height << 16
};
static_assert(sizeof(Rec) == 80, "Rec layout");
constexpr int kRecGroups = 5;  // 16-B field groups (the 80 B of the record)
constexpr uint32_t kTexAlign = 16;   // texture offsets (texels) are multiples of this: Rec::atex packing
__host__ __device__ inline uint32_t rec_atex(uint32_t offset, uint32_t thr) { return (offset / kTexAlign) | (thr << 24); }

struct FrameDev {                // csg_frame mirror
  float view[16];
  float proj[16];
  uint32_t xform_set;
  uint32_t frame_id;
  uint32_t records_hint;         // raster records measured by csg_size_work (0: not measured)
  uint32_t bins_hint;            // tile-bin entries measured likewise
};

// A frame's region of the launch chain's record and bin pools (k_plan): the
// records [rec_base, rec_base + rec_cap) of `recs` / `rect`, the bin entries
// [bin_base, bin_base + bin_cap) of `bins`.  Bases are multiples of 4 records
// (16-B aligned rect rows: k_count / k_bin load 4 at once).
struct Slab {
  uint64_t rec_base, bin_base;
  uint32_t rec_cap, bin_cap;
  uint32_t pad[2];
};
static_assert(sizeof(Slab) == 32, "Slab layout");

// Geometry is stored de-indexed ("triangle soup"): the authored vertex and
// index arrays are expanded at upload so a triangle is one contiguous 36-B
// (positions) / 24-B (uvs) record.  World2 has ~2 vertices per triangle, so
// the soup is the same size as the indexed arrays (12 B/vertex + 12 B/tri)
// while removing the dependent index->vertex loads from k_setup and resolve.
struct SceneDev {
  const float* tri_pos;        // [T][3][3] object space
  const float* tri_uv;         // [T][3][2] (zeros for meshes without uvs)
  const InstDesc* inst;        // [I]
  const TexDesc* texd;
  const uint8_t* texels;        // RGBA8, all textures back to back (TexDesc.offset in texels)
  const uint32_t* aquad;        // alpha quads, same indexing (see alpha_pass)
  const uint32_t* acls;         // 2-bit alpha-test class per alpha quad, 16 per word (see alpha_pass)
  uint32_t n_inst;
  uint32_t W, H, tiles_x, tiles_y, n_tiles;
  float near_clip, far_clip;
  float inv_near, inv_far;     // 1/near_clip, 1/far_clip (IEEE, computed on the host)
  uint32_t dbg;                // ablation switches (CSG_DEBUG; 0 in production)
  // Kernel uids are (instance << uid_shift) | (soup index of the triangle):
  // the same order as the spec's (instance << 20) | mesh triangle (within an
  // instance the soup index is the mesh's base plus the triangle), and the
  // resolve finds the triangle without loading the instance first.
  uint32_t uid_shift;
  uint32_t rect_ys;            // tile rectangles hold tile-row pairs (1: more than 256 tile rows) or rows (0)
};

// Bits of overflow[0] (sticky until csg_synchronize / csg_render_batch reads them)
constexpr uint32_t kOvRecords = 1u;      // a frame emitted more raster records than its slab holds
constexpr uint32_t kOvBins = 2u;         // a frame's tile-bin entries exceeded its slab
constexpr uint32_t kOvBadSet = 4u;       // device frame named a transform set >= n_sets (rendered with set 0)
constexpr uint32_t kOvBadKpSet = 8u;     // device frame named a keypoint set >= n_kp_sets (keypoints vis 0)

struct BatchDev {
  const FrameDev* frames;      // [F]
  uint32_t* fset;              // [F] the frame's transform set, range-checked by k_clip (every later kernel reads this)
  uint32_t n_sets;             // transform sets resident (models / mats / lights tables)
  uint32_t n_kp_sets;          // keypoint sets resident
  const float* models;         // [n_sets][I][16]
  const MatDesc* mats;         // [n_sets][n_mat] materials with the set's texture swaps applied
  const InstSetDev* iset;      // [n_sets][n_inst] each instance's resolved material per set
  const LightDev* lights;      // [n_sets]
  uint32_t n_mat;
  float* clip;                 // [F][I][12] rows 0,1,3 of P*V*M
  float* pv;                   // [F][12]    rows 0,1,3 of P*V
  Rec* recs;                   // record pool: frame f's records at slab[f].rec_base
  uint32_t* rect;              // same indexing: tile rect tx0|ty0<<8|tx1<<16|ty1<<24
  const Slab* slab;            // [F] each frame's region of the pools (k_plan)
  uint32_t* rec_count;         // [F * kCounterStride] (one cache line per frame: no atomic contention)
  uint32_t* tile_count;        // [F][n_tiles] (k_colscan)
  uint32_t* tile_off;          // [F][n_tiles+1]
  uint32_t* bins;              // bin pool: frame f's tile lists at slab[f].bin_base (tile_off relative to it)
  uint32_t* bcount;            // [F][bin_blocks][n_tiles]: each k_count block's tile counts,
                               //   then (k_colscan) the block's first slot in each tile's list, tile-relative
  uint32_t bin_blocks;
  uint32_t* overflow;          // [16]: [0] bit0 rec, bit1 bins; [1..] profiling counters (CSG_DEBUG 512)
  // outputs (device)
  uint8_t* rgb;                // [F][H][W][3] or null
  int32_t* inst;               // [F][H][W] or null
  float* depth;                // [F][H][W] or null
  uint16_t* normals;           // [F][H][W][3] f16 bits or null
  float* points;               // [F][H][W][3] world xyz (NaN: no hit) or null
  float* cam;                  // [F][kCamFloats] camera-to-world rotation, position, fx fy cx cy
  uint32_t* stats;             // [F][n_labels][5] or null
  uint32_t* covered;           // [F][n_labels] unoccluded pixels per label (k_raster<true> only), bit 31: unknown
  uint32_t n_labels;
  const float* kp;             // [n_sets][K][3]
  uint32_t n_kp;
  float* kp_uv;                // [F][K][2]
  int32_t* kp_vis;             // [F][K]
  float* kp_w;                 // [F][K] camera-space w (distance to the image plane)
  uint32_t* kp_pix;            // [F][K] px | py << 16 of in-view keypoints, else ~0
  uint32_t* kp_tiles;          // [F][tile_words] bitmap of tiles holding an in-view keypoint
  uint32_t tile_words;
  uint32_t* drange;            // [2][drange_F] min / max bits of the valid depths of each frame, reduced by
  uint32_t drange_F;           //   k_raster's resolve (null: not wanted)
  uint32_t dbg;                // ablation switches for profiling only (CSG_DEBUG env; 0 in production)
  uint32_t px_align;           // (first pixel of this launch chain in the output buffers) mod 4
};

// launchers (all enqueue on `st`)
// k_plan: each frame's slab from its hints (use_hints; 0 = none) or the
// default caps, packed back to back; frames past a pool's end get what is
// left (possibly nothing: they overflow).  need[0], need[1]: raised to the
// pool entries the chain asked for (a running maximum over the batch's
// chains).  Pools are multiples of 4 entries.
void launch_plan(const FrameDev* frames, uint32_t F, uint32_t def_rec, uint32_t def_bin, uint64_t rec_pool,
                 uint64_t bin_pool, int use_hints, Slab* slab, uint64_t* need, hipStream_t st);
// csg_size_work's hint for a measured count: count x (1 + margin) + pad, 4-aligned, < 2^31
inline uint32_t hinted_cap(uint32_t count, double margin, uint32_t pad) {
  const double c = (double)count * (1.0 + margin);
  const uint64_t v = (uint64_t)c + (c > (double)(uint64_t)c ? 1u : 0u) + pad;
  return (uint32_t)(((v < 0x7FFFFFF0ull ? v : 0x7FFFFFF0ull) + 3u) & ~3ull);
}
void launch_clip(const SceneDev& s, const BatchDev& b, uint32_t F, hipStream_t st);
void launch_setup(const SceneDev& s, const BatchDev& b, const Chunk* chunks, uint32_t n_chunks,
                  uint32_t F, hipStream_t st);
void launch_count(const SceneDev& s, const BatchDev& b, uint32_t F, uint32_t blocks, hipStream_t st);
void launch_scan(const SceneDev& s, const BatchDev& b, uint32_t F, hipStream_t st);
void launch_colscan(const SceneDev& s, const BatchDev& b, uint32_t F, hipStream_t st);
void launch_bin(const SceneDev& s, const BatchDev& b, uint32_t F, uint32_t blocks, hipStream_t st);
void launch_raster(const SceneDev& s, const BatchDev& b, uint32_t F, hipStream_t st);
// depth visualisation (GDP:1690-1709): from the per-frame min / max of the valid
// depth that k_raster reduced (range [2][F] as float bits: row 0 min, row 1 max),
// the JET-coloured RGB8 image; lut = 256 packed r | g << 8 | b << 16
void launch_depth_vis(const float* depth, uint32_t npx, uint32_t F, const uint32_t* range, const uint32_t* lut,
                      uint8_t* vis, float* range_out, hipStream_t st);
void launch_init_stats(const BatchDev& b, uint32_t F, hipStream_t st);
void launch_keypoints(const SceneDev& s, const BatchDev& b, uint32_t F, hipStream_t st);
void launch_inst_bounds(const SceneDev& s, const Chunk* chunks, uint32_t n_chunks, const float* models,
                        uint32_t* out, hipStream_t st);
void launch_project(const float* pts, uint32_t n, const float* pv12, float W, float H, float near_clip,
                    float* uv, int32_t* vis, hipStream_t st);
// ids [lo, hi) of the int32 instance image as (id + 1) in `bytes` (1 or 2) bytes (the host wire)
void launch_narrow_ids(const int32_t* src, size_t lo, size_t hi, uint32_t bytes, void* dst, hipStream_t st);

}  // namespace csg
