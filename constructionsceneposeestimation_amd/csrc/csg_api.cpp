// C-ABI host side of libcsg.so (see include/csg_api.h).
//
// Owns the device copy of the scene (one HBM-resident scene per context,
// shared by every frame of every batch), the per-batch work buffers sized
// for `max_frames`, and the launch sequence of csg_kernels.hip.  All
// validation that protects the GPU from out-of-bounds indices happens here,
// on the host, before anything is uploaded.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cstddef>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <memory>
#include <string>
#include <vector>

#include "../../include/csg_api.h"
#include "csg_encode.h"
#include "csg_kernels.h"
#include "csg_widen.h"

using namespace csg;

namespace {

// A device allocation owned by one object: freed by release() or at the end
// of its scope (a local scratch buffer cannot leak on an early error return).
template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  hipError_t alloc(size_t count) {
    if (count <= n && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    if (count == 0) return hipSuccess;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&p), count * sizeof(T));
    if (e == hipSuccess) n = count;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

// Default frames per launch chain: the whole batch.  Measured on C3 (1080p,
// 60 frames): chains of 2/4/8/20 frames cost 3.7x/2.0x/1.6x/1.3x the time of
// one chain -- per-launch tails and k_setup's early-exit blocks dominate, and
// keeping records in the Infinity Cache does not pay that back.  Smaller
// chains only bound the work-buffer memory.
constexpr uint32_t kAutoChainFrames = 0xFFFFFFFFu;

// Transform / keypoint / randomisation sets per context (ids 0..kMaxSets-1;
// the tables hold max id + 1 sets).  The bench's default run at 2,880
// frames per step uses 7,200 epochs on one rank.
constexpr uint32_t kMaxSets = 65536;

struct HostTexture {
  std::vector<uint8_t> rgba;
  uint32_t w = 0, h = 0;
  bool present = false;
};

}  // namespace

struct csg_ctx {
  csg_config cfg{};
  std::string err;
  hipStream_t stream = nullptr;
  uint32_t tiles_x = 0, tiles_y = 0, n_tiles = 0;

  // scene
  bool have_scene = false;
  uint32_t n_inst = 0, n_meshes = 0, n_materials = 0;
  uint64_t n_tris_total = 0;
  DevBuf<float> tri_pos, tri_uv;       // de-indexed triangle soup (see SceneDev)
  DevBuf<InstDesc> inst;
  std::vector<MatDesc> h_mats;
  std::vector<MatDesc> h_set_mats;      // [sets][n_materials] as uploaded
  std::vector<MeshDesc> h_meshes;
  DevBuf<Chunk> chunks;
  uint32_t n_chunks = 0;
  uint32_t uid_shift = kUidShift;       // SceneDev::uid_shift
  std::vector<HostTexture> textures;
  bool tex_dirty = true;
  DevBuf<uint8_t> texels;
  DevBuf<uint32_t> aquad;
  DevBuf<uint32_t> acls;                // alpha-test class of each alpha quad (see build_alpha_classes)
  std::vector<int> acls_thr;            // per texture: the threshold acls was built for
  DevBuf<TexDesc> texd;
  LightDev light{{0.26f, 0.29f, 0.34f}, {0.78f, 0.78f, 0.78f}, {0.7071f, 0.f, 0.7071f},
                 191u | (217u << 8) | (255u << 16)};   // default (csg_set_light)
  // domain randomisation per transform set (csg_set_dr_light / csg_set_dr_textures)
  std::vector<LightDev> dr_light;
  std::vector<uint8_t> dr_light_valid;
  std::vector<int32_t> dr_tex;          // [sets][n_materials]; kKeepTexture = the material's own
  bool dr_dirty = true;
  DevBuf<LightDev> lights;
  DevBuf<MatDesc> set_mats;
  uint32_t n_table_sets = 0;
  std::vector<float> h_models;          // [sets][I][16]
  std::vector<uint8_t> set_valid;
  DevBuf<float> models;
  bool models_dirty = true;
  uint32_t n_kp = 0;
  std::vector<float> h_kp;              // [sets][K][3]
  std::vector<uint8_t> kp_valid;
  DevBuf<float> kp;
  bool kp_dirty = true;

  // per-batch work buffers: record and bin pools shared by the frames of a
  // launch chain, each frame's region (Slab) planned by k_plan from its hints
  // or the per-frame caps rec_cap / bin_cap
  uint32_t rec_cap = 0, bin_cap = 0, work_frames = 0;
  uint64_t rec_pool = 0, bin_pool = 0;            // pool entries allocated
  bool use_hints = false;                         // csg_size_work sized the pools from frame hints
  uint32_t hint_fallbacks = 0;                    // re-renders the hinted pools caused (csg_work_info)
  uint64_t plan_rec_pool = 0, plan_bin_pool = 0;  // ... to these
  DevBuf<Slab> slab;                              // [chain frames] (k_plan)
  DevBuf<uint64_t> plan_need;                     // [2] pool entries the batch's largest chain asked for (k_plan)
  DevBuf<FrameDev> frames;
  // Pinned staging ring for host frame records: a batch's records are copied
  // into the next slot, and a slot is reused only after the H2D copy that read
  // it has completed (its event), so back-to-back async batches never render
  // each other's cameras.
  static constexpr uint32_t kStaging = 4;
  FrameDev* h_stage[kStaging] = {};
  hipEvent_t stage_ev[kStaging] = {};
  bool stage_busy[kStaging] = {};
  uint32_t stage_next = 0;
  // The stream of the most recent enqueue.  The work buffers are shared, so a
  // batch on a different stream first waits for the previous stream to drain;
  // csg_synchronize waits on it.
  hipStream_t last_stream = nullptr;
  DevBuf<uint32_t> fset;                // [chain frames] checked transform set of each frame (k_clip)
  DevBuf<float> clip, pv;
  DevBuf<Rec> recs;
  DevBuf<uint32_t> rect, rec_count, tile_count, tile_off, bins, overflow;
  DevBuf<uint32_t> bcount;              // [chain frames][bin_blocks][n_tiles] count grid
  DevBuf<InstSetDev> iset;              // [n_table_sets][n_inst] resolved materials (sync_scene_state)
  std::vector<InstDesc> h_inst;         // host copy of the instance table
  // internal outputs (host-output mode / scratch)
  DevBuf<uint8_t> o_rgb;
  DevBuf<int32_t> o_inst;
  DevBuf<float> o_depth, o_kp_uv, kp_w, o_points, cam;
  DevBuf<uint16_t> o_normals;
  DevBuf<int32_t> o_kp_vis;
  DevBuf<uint32_t> kp_pix, kp_tiles;
  DevBuf<uint32_t> o_stats;
  DevBuf<uint8_t> o_dvis;               // depth visualisation (host-output mode)
  DevBuf<float> o_drange;
  DevBuf<uint32_t> o_cov;               // label coverage (host-output mode)
  DevBuf<uint32_t> drange;              // [2][chain frames] min / max depth bits (k_raster's resolve)
  DevBuf<uint32_t> jet;                 // JET colour map, 256 x (r | g << 8 | b << 16)
  // images of the last batch (for the file encoders) and the encoders' buffers
  const uint8_t* last_rgb = nullptr;
  const float* last_depth = nullptr;
  const float* last_points = nullptr;
  const uint8_t* last_dvis = nullptr;
  DevBuf<EncPng> enc_rgb, enc_dpng;
  DevBuf<uint2> enc_rowsum;
  DevBuf<uint32_t> enc_rows_rgb, enc_rows_dpng, enc_rows_csv, enc_rows_pcd;
  DevBuf<uint64_t> enc_fsize, enc_foff, enc_zoff;
  DevBuf<uint8_t> enc_zbuf, enc_out;
  DevBuf<uint8_t> dstat_part;           // depth-statistics partial sums
  DevBuf<double> o_dstats;              // depth statistics (host-output mode)
  uint64_t enc_total = 0;               // bytes of the last batch's files (0: none)
  uint32_t enc_nfiles = 0;
  std::vector<uint64_t> h_foff;

  // timing: ring of per-batch event quintuples (recorded, never waited on in the loop)
  bool timing = true;
  static constexpr uint32_t kRing = 4096;
  std::vector<hipEvent_t> ring;         // kRing * 5
  std::vector<uint32_t> ring_frames;
  uint64_t ring_count = 0;
  hipEvent_t* ev = nullptr;             // events of the most recent batch
  uint32_t last_F = 0;
  uint32_t dbg = 0;                     // CSG_DEBUG ablation bits (profiling builds of the pipeline only)
  // k_count / k_bin workgroups per frame (CSG_BINBLOCKS: A/B only; set in
  // csg_create from the tile count).  16 at 1080p's 4,080 tiles of 32 x 16
  // keeps the [blocks][tiles] count grid the size 32 blocks gave 32 x 32 tiles
  // (C3: binning 2.27 vs 2.69 ms per 960 frames with 16 vs 32 blocks; at 2,880
  // frames per step 8 / 16 / 24 blocks: binning 5.8 / 6.2 / 6.3 ms, k_raster
  // 97.3 / 97.1 / 96.9 ms); 8 above 8,192 tiles (C5 at 4K, 16,200 tiles, 480
  // frames: binning 4.3 / 4.7 / 4.4 / 5.2 ms with 8 / 16 / 4 / 2 blocks;
  // profiles/r05/ab/tile_shape.md)
  uint32_t bin_blocks = 32;
  uint32_t chain_frames = 0;            // frames per launch chain (cfg.frames_per_launch; CSG_CHAIN overrides)
  // Host outputs: each launch chain's slice is copied to the host on copy_stream
  // while the next chains render (created with the first host-output batch).
  static constexpr uint32_t kCopyEv = 16;
  hipStream_t copy_stream = nullptr;
  hipEvent_t copy_ev[kCopyEv] = {};
  hipEvent_t copy_done = nullptr;
  // The host wire of the instance ids (csg_widen.h): a host-output batch's ids
  // cross PCIe as (id + 1) in ids_bytes (1 with at most 255 labels, 2 with at
  // most 65,535; 4 = int32 as rendered, no narrowing) and are widened to the
  // caller's int32 by WidenPool threads while later chains render.
  // CSG_NARROW_IDS=0 keeps int32 on the wire (A/B, tests).
  uint32_t ids_bytes = 4;               // set by csg_upload_scene from the label range
  bool narrow_ids = true;
  bool split_pageable = true;           // CSG_SPLIT_PAGEABLE=0: pageable host outputs as one chain (A/B, tests)
  DevBuf<uint8_t> o_ids_n;              // [F][H][W] narrowed ids (device)
  uint8_t* h_ids_n = nullptr;           // ... their pinned host landing buffer
  size_t h_ids_n_bytes = 0;
  // the last sizing pass (csg_size_work)
  uint32_t sized_frames = 0, sized_max_rec = 0, sized_max_bin = 0;
  double sized_mean_rec = 0.0, sized_mean_bin = 0.0;

  int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    err = buf;
    return code;
  }
};

#define HIP_TRY(ctx, expr)                                                                           \
  do {                                                                                               \
    hipError_t _e = (expr);                                                                          \
    if (_e != hipSuccess)                                                                            \
      return (ctx)->fail(_e == hipErrorOutOfMemory ? CSG_ERR_OOM : CSG_ERR_DEVICE, "%s: %s", #expr,  \
                         hipGetErrorString(_e));                                                     \
  } while (0)

// Wait for everything this context enqueued, on its own stream and on the
// caller's stream of the most recent batch.
static int drain(csg_ctx* c) {
  if (c->last_stream && c->last_stream != c->stream) HIP_TRY(c, hipStreamSynchronize(c->last_stream));
  if (c->stream) HIP_TRY(c, hipStreamSynchronize(c->stream));
  return CSG_OK;
}

// Read the sticky overflow / error word of every batch since it was last
// read, clear it, and turn it into a status.  Callers have drained the streams.
static int take_flags(csg_ctx* c, uint32_t* flags_out) {
  uint32_t ov = 0;
  HIP_TRY(c, hipMemcpy(&ov, c->overflow.p, 4, hipMemcpyDeviceToHost));
  if ((c->dbg & 512u)) {   // profiling counters, cumulative since the context was created
    uint32_t ctr[16];
    HIP_TRY(c, hipMemcpy(ctr, c->overflow.p, sizeof(ctr), hipMemcpyDeviceToHost));
    fprintf(stderr, "[csg] staged_recs %u row_items %u spans %u l2_items %u alpha_fail %u alpha_pass %u early_z %u "
            "wide_rows %u small_recs %u small_rows %u small_items %u alpha_waves %u alpha_wave_lanes %u l2_waves %u "
            "l2_wave_lanes %u\n", ctr[1], ctr[2], ctr[3], ctr[4], ctr[5], ctr[6], ctr[7], ctr[8], ctr[9], ctr[10],
            ctr[11], ctr[12], ctr[13], ctr[14], ctr[15]);
  }
  if (flags_out) *flags_out = ov;
  if (!ov) return CSG_OK;
  // cleared on the context stream and waited for: the next batch (on any
  // stream) is enqueued only after the clear has landed
  HIP_TRY(c, hipMemsetAsync(c->overflow.p, 0, 4, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  if (ov & (kOvBadSet | kOvBadKpSet))
    return c->fail(CSG_ERR_INVALID,
                   "device frame records named a transform set >= %u or a keypoint set >= %u (flags %u); those "
                   "frames rendered with set 0 / without keypoints",
                   (unsigned)c->set_valid.size(), (unsigned)c->kp_valid.size(), ov);
  return c->fail(CSG_ERR_OVERFLOW, "work buffer overflow (flags %u): records_per_frame=%u bins_per_frame=%u", ov,
                 c->rec_cap, c->bin_cap);
}

// OpenCV's COLORMAP_JET (the reference's cv2.applyColorMap, GDP:1703): the
// GNU Octave "jet" map sampled at x = k/255, stored as float, scaled by 255
// in float and rounded half to even (Mat::convertTo to CV_8U).  OpenCV is not
// in this image, so the table is a restatement, not a copy.
static void jet_lut(uint32_t* lut) {
  for (int k = 0; k < 256; ++k) {
    const double x = (double)k / 255.0;
    const double r = (x >= 3.0 / 8 && x < 5.0 / 8) ? 4 * x - 1.5 : (x >= 5.0 / 8 && x < 7.0 / 8) ? 1.0
                     : (x >= 7.0 / 8) ? -4 * x + 4.5 : 0.0;
    const double g = (x >= 1.0 / 8 && x < 3.0 / 8) ? 4 * x - 0.5 : (x >= 3.0 / 8 && x < 5.0 / 8) ? 1.0
                     : (x >= 5.0 / 8 && x < 7.0 / 8) ? -4 * x + 3.5 : 0.0;
    const double b = (x < 1.0 / 8) ? 4 * x + 0.5 : (x >= 1.0 / 8 && x < 3.0 / 8) ? 1.0
                     : (x >= 3.0 / 8 && x < 5.0 / 8) ? -4 * x + 2.5 : 0.0;
    const double ch[3] = {r, g, b};
    uint32_t v = 0;
    for (int c = 0; c < 3; ++c) {
      const float p = (float)ch[c] * 255.0f;
      const long q = std::lrint(p);   // default rounding mode: nearest, ties to even
      v |= (uint32_t)std::min(255L, std::max(0L, q)) << (8 * c);
    }
    lut[k] = v;
  }
}

extern "C" {

int csg_abi_version(void) { return CSG_ABI_VERSION; }

const char* csg_last_error(const csg_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int csg_create(const csg_config* cfg, csg_ctx** out) {
  if (!cfg || !out) return CSG_ERR_INVALID;
  *out = nullptr;
  // tile rectangles carry 8-bit tile coordinates (k_setup's rect, k_count / k_bin): at most 256 tile columns
  // and 512 tile rows (rows in pairs above 256: 8,192 x 8,192 px at 32 x 16 tiles)
  if (cfg->width == 0 || cfg->height == 0 || cfg->width > 256u * kTileW || cfg->height > 512u * kTileH ||
      cfg->max_frames == 0 ||
      !(cfg->near_clip >= 0x1p-126f) || !(cfg->far_clip > cfg->near_clip) || !(cfg->far_clip <= 0x1p126f))
    return CSG_ERR_INVALID;   // clip distances in [2^-126, 2^126]: the range of rcp_ieee's proof (k_setup, k_raster)
  csg_ctx* c = new csg_ctx();
  c->cfg = *cfg;
  if (const char* d = getenv("CSG_DEBUG")) c->dbg = (uint32_t)strtoul(d, nullptr, 0);
  if (const char* v = getenv("CSG_NARROW_IDS")) c->narrow_ids = atoi(v) != 0;
  if (const char* v = getenv("CSG_SPLIT_PAGEABLE")) c->split_pageable = atoi(v) != 0;
  c->chain_frames = cfg->frames_per_launch ? cfg->frames_per_launch : kAutoChainFrames;
  if (const char* v = getenv("CSG_CHAIN")) c->chain_frames = (uint32_t)std::max(1, atoi(v));
  c->chain_frames = std::min(c->chain_frames, cfg->max_frames);
  c->tiles_x = (cfg->width + kTileW - 1) / kTileW;
  c->tiles_y = (cfg->height + kTileH - 1) / kTileH;
  c->n_tiles = c->tiles_x * c->tiles_y;
  c->bin_blocks = kTileH >= 32 ? 32u : (c->n_tiles > 8192u ? 8u : 16u);
  if (const char* v = getenv("CSG_BINBLOCKS")) c->bin_blocks = std::max(1, std::min(1024, atoi(v)));
  hipError_t e = hipSetDevice(cfg->device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  c->ring.assign((size_t)csg_ctx::kRing * 5, nullptr);
  c->ring_frames.assign(csg_ctx::kRing, 0);
  for (size_t k = 0; k < c->ring.size() && e == hipSuccess; ++k) e = hipEventCreate(&c->ring[k]);
  for (uint32_t k = 0; k < csg_ctx::kStaging && e == hipSuccess; ++k)
    e = hipEventCreateWithFlags(&c->stage_ev[k], hipEventDisableTiming);
  // the overflow / error word lives as long as the context: it is sticky across
  // asynchronous batches and cleared only when csg_synchronize or
  // csg_render_batch has read it
  if (e == hipSuccess) e = c->overflow.alloc(16);
  if (e == hipSuccess) e = hipMemset(c->overflow.p, 0, 16 * sizeof(uint32_t));
  if (e == hipSuccess) e = c->jet.alloc(256);
  if (e == hipSuccess) {
    uint32_t lut[256];
    jet_lut(lut);
    e = hipMemcpy(c->jet.p, lut, sizeof(lut), hipMemcpyHostToDevice);
  }
  c->ev = c->ring.data();
  if (e != hipSuccess) {
    c->err = hipGetErrorString(e);
    csg_destroy(c);
    return CSG_ERR_DEVICE;
  }
  *out = c;
  return CSG_OK;
}

void csg_destroy(csg_ctx* c) {
  if (!c) return;
  if (c->last_stream && c->last_stream != c->stream) (void)hipStreamSynchronize(c->last_stream);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  // (every batch's stream waits for its copies and id widening on the copy
  // stream, copy_done; synchronized here too before the buffers they read go)
  if (c->copy_stream) (void)hipStreamSynchronize(c->copy_stream);
  c->tri_pos.release(); c->tri_uv.release(); c->inst.release(); c->set_mats.release(); c->iset.release(); c->lights.release();
  c->chunks.release();
  c->texels.release();
  c->aquad.release();
  c->acls.release();
  c->texd.release(); c->models.release(); c->kp.release(); c->frames.release(); c->clip.release();
  c->pv.release(); c->recs.release(); c->rect.release(); c->rec_count.release(); c->tile_count.release();
  c->slab.release(); c->plan_need.release();
  c->tile_off.release(); c->bins.release(); c->bcount.release(); c->overflow.release(); c->o_rgb.release();
  c->o_inst.release(); c->o_depth.release(); c->o_kp_uv.release(); c->o_kp_vis.release(); c->o_stats.release();
  c->kp_w.release(); c->kp_pix.release(); c->kp_tiles.release();
  c->o_points.release(); c->o_normals.release(); c->cam.release(); c->fset.release();
  c->o_dvis.release(); c->o_drange.release(); c->o_cov.release(); c->drange.release(); c->jet.release();
  for (uint32_t k = 0; k < csg_ctx::kStaging; ++k) {
    if (c->h_stage[k]) (void)hipHostFree(c->h_stage[k]);
    if (c->stage_ev[k]) (void)hipEventDestroy(c->stage_ev[k]);
  }
  for (auto& e : c->ring)
    if (e) (void)hipEventDestroy(e);
  if (c->h_ids_n) (void)hipHostFree(c->h_ids_n);
  c->o_ids_n.release();
  for (auto& e : c->copy_ev)
    if (e) (void)hipEventDestroy(e);
  if (c->copy_done) (void)hipEventDestroy(c->copy_done);
  if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

int csg_upload_scene(csg_ctx* c, const csg_mesh* meshes, uint32_t n_meshes, const csg_material* materials,
                     uint32_t n_materials, const csg_instance* inst, uint32_t n_inst) {
  if (!c) return CSG_ERR_INVALID;
  if (!meshes || !materials || !inst || n_meshes == 0 || n_materials == 0 || n_inst == 0)
    return c->fail(CSG_ERR_INVALID, "upload_scene: empty scene");
  if (n_inst >= kMaxInstances) return c->fail(CSG_ERR_LIMIT, "upload_scene: %u instances >= %u", n_inst, kMaxInstances);
  HIP_TRY(c, hipSetDevice(c->cfg.device));
  {  // batches in flight read the scene and the work buffers this replaces
    const int rc = drain(c);
    if (rc) return rc;
  }
  std::vector<float> pos, uvs;
  std::vector<uint32_t> tris, uvt;
  std::vector<MeshDesc> md(n_meshes);
  for (uint32_t m = 0; m < n_meshes; ++m) {
    const csg_mesh& M = meshes[m];
    if (M.n_tris >= kMaxTrisPerMesh) return c->fail(CSG_ERR_LIMIT, "mesh %u: %u tris >= 2^20", m, M.n_tris);
    if (M.material >= n_materials) return c->fail(CSG_ERR_INVALID, "mesh %u: material %u out of range", m, M.material);
    if ((M.n_vertices && !M.positions) || (M.n_tris && !M.indices))
      return c->fail(CSG_ERR_INVALID, "mesh %u: null arrays", m);
    for (uint64_t k = 0; k < 3ull * M.n_tris; ++k)
      if (M.indices[k] >= M.n_vertices) return c->fail(CSG_ERR_INVALID, "mesh %u: index out of range", m);
    const bool has_uv = M.uvs && M.uv_indices && M.n_uvs;
    if (has_uv)
      for (uint64_t k = 0; k < 3ull * M.n_tris; ++k)
        if (M.uv_indices[k] >= M.n_uvs) return c->fail(CSG_ERR_INVALID, "mesh %u: uv index out of range", m);
    md[m] = MeshDesc{(uint32_t)(pos.size() / 3), (uint32_t)(tris.size() / 3), M.n_tris, (uint32_t)(uvs.size() / 2),
                     has_uv ? 1u : 0u, M.material};
    pos.insert(pos.end(), M.positions, M.positions + 3ull * M.n_vertices);
    tris.insert(tris.end(), M.indices, M.indices + 3ull * M.n_tris);
    if (has_uv) {
      uvs.insert(uvs.end(), M.uvs, M.uvs + 2ull * M.n_uvs);
      uvt.insert(uvt.end(), M.uv_indices, M.uv_indices + 3ull * M.n_tris);
    } else {
      uvt.insert(uvt.end(), 3ull * M.n_tris, 0u);
    }
  }
  if (uvs.empty()) uvs.assign(2, 0.f);
  std::vector<MatDesc> mats(n_materials);
  for (uint32_t k = 0; k < n_materials; ++k) {
    if (materials[k].alpha_threshold > 255u)
      return c->fail(CSG_ERR_INVALID, "material %u: alpha_threshold %u > 255 (alpha is 8-bit)", k,
                     materials[k].alpha_threshold);
    memcpy(mats[k].base, materials[k].base_color, 4);
    mats[k].texture = materials[k].texture;
    mats[k].alpha_test = materials[k].alpha_test;
    mats[k].alpha_threshold = materials[k].alpha_threshold;
  }
  // de-index: one 9-float position record and one 6-float uv record per triangle
  const size_t n_soup = tris.size() / 3;
  {  // kernel uids: instance << uid_shift | soup index (SceneDev::uid_shift)
    uint32_t shift = kUidShift;
    while (shift < 31 && (1ull << shift) < n_soup) ++shift;
    if ((1ull << shift) < n_soup || (uint64_t)n_inst > (1ull << (32 - shift)))
      return c->fail(CSG_ERR_LIMIT, "upload_scene: %zu soup triangles x %u instances exceed 32-bit uids", n_soup, n_inst);
    c->uid_shift = shift;
  }
  std::vector<float> tri_pos(n_soup * 9), tri_uv(n_soup * 6, 0.f);
  for (uint32_t m = 0; m < n_meshes; ++m) {
    const MeshDesc& d = md[m];
    for (uint32_t t = 0; t < d.ntris; ++t) {
      const size_t g = (size_t)d.tbase + t;
      for (int k = 0; k < 3; ++k) {
        memcpy(&tri_pos[g * 9 + 3 * k], &pos[((size_t)d.vbase + tris[g * 3 + k]) * 3], 3 * sizeof(float));
        if (d.has_uv) memcpy(&tri_uv[g * 6 + 2 * k], &uvs[((size_t)d.uvbase + uvt[g * 3 + k]) * 2], 2 * sizeof(float));
      }
    }
  }
  std::vector<InstDesc> idesc(n_inst);
  std::vector<Chunk> ch;
  std::vector<float> models((size_t)n_inst * 16);
  uint64_t ntot = 0;
  for (uint32_t i = 0; i < n_inst; ++i) {
    if (inst[i].mesh >= n_meshes) return c->fail(CSG_ERR_INVALID, "instance %u: mesh out of range", i);
    const MeshDesc& mi = md[inst[i].mesh];
    idesc[i] = InstDesc{mi.tbase, mi.material, mi.has_uv, inst[i].inst_idx};
    memcpy(&models[(size_t)i * 16], inst[i].model, 16 * sizeof(float));
    const uint32_t nt = md[inst[i].mesh].ntris;
    const MeshDesc& md_i = md[inst[i].mesh];
    for (uint32_t s0 = 0; s0 < nt; s0 += kBlock) {
      Chunk c0{};
      c0.inst = i;
      c0.start = s0;
      c0.count = std::min<uint32_t>(kBlock, nt - s0);
      c0.soup = md_i.tbase + s0;   // soup index of the chunk's first triangle
      for (int a = 0; a < 3; ++a) { c0.lo[a] = INFINITY; c0.hi[a] = -INFINITY; }
      for (uint32_t t = s0; t < s0 + c0.count; ++t)
        for (int k = 0; k < 3; ++k) {
          const float* p = &pos[((size_t)md_i.vbase + tris[((size_t)md_i.tbase + t) * 3 + k]) * 3];
          for (int a = 0; a < 3; ++a) { c0.lo[a] = std::min(c0.lo[a], p[a]); c0.hi[a] = std::max(c0.hi[a], p[a]); }
        }
      ch.push_back(c0);
    }
    ntot += nt;
  }
  if (ch.empty()) return c->fail(CSG_ERR_INVALID, "upload_scene: no triangles");
  HIP_TRY(c, c->tri_pos.alloc(std::max<size_t>(tri_pos.size(), 9)));
  HIP_TRY(c, c->tri_uv.alloc(std::max<size_t>(tri_uv.size(), 6)));
  HIP_TRY(c, c->inst.alloc(n_inst));
  HIP_TRY(c, c->chunks.alloc(ch.size()));
  HIP_TRY(c, hipMemcpy(c->tri_pos.p, tri_pos.data(), tri_pos.size() * 4, hipMemcpyHostToDevice));
  HIP_TRY(c, hipMemcpy(c->tri_uv.p, tri_uv.data(), tri_uv.size() * 4, hipMemcpyHostToDevice));
  HIP_TRY(c, hipMemcpy(c->inst.p, idesc.data(), idesc.size() * sizeof(InstDesc), hipMemcpyHostToDevice));
  c->h_inst = idesc;
  {   // the ids the resolve writes are instance labels and -1: the narrowest host wire for them
    int32_t lo = -1, hi = -1;
    for (const InstDesc& d : idesc) { lo = std::min(lo, d.label); hi = std::max(hi, d.label); }
    c->ids_bytes = lo < -1 ? 4u : hi <= 254 ? 1u : hi <= 65534 ? 2u : 4u;
  }
  c->iset.release();   // rebuilt for the new instances by the next sync_scene_state
  HIP_TRY(c, hipMemcpy(c->chunks.p, ch.data(), ch.size() * sizeof(Chunk), hipMemcpyHostToDevice));
  c->n_inst = n_inst;
  c->n_meshes = n_meshes;
  c->n_materials = n_materials;
  c->h_mats = mats;
  c->h_meshes = md;
  c->n_chunks = (uint32_t)ch.size();
  c->n_tris_total = ntot;
  c->h_models = models;
  c->set_valid.assign(1, 1);
  c->models_dirty = true;
  c->dr_tex.clear();
  c->dr_dirty = true;
  c->h_kp.clear();
  c->kp_valid.clear();
  c->n_kp = 0;
  c->kp_dirty = true;
  c->have_scene = true;
  c->work_frames = 0;  // re-size work buffers,
  c->rec_cap = 0;      // with caps derived from this scene (or the config's fixed ones)
  c->bin_cap = 0;
  return CSG_OK;
}

int csg_upload_texture(csg_ctx* c, uint32_t tex_id, const uint8_t* rgba8, uint32_t w, uint32_t h) {
  if (!c) return CSG_ERR_INVALID;
  if (!rgba8 || w == 0 || h == 0 || w > 16384 || h > 16384 || tex_id >= 4096)
    return c->fail(CSG_ERR_INVALID, "upload_texture: bad arguments");
  if (c->textures.size() <= tex_id) c->textures.resize(tex_id + 1);
  HostTexture& t = c->textures[tex_id];
  t.rgba.assign(rgba8, rgba8 + (size_t)w * h * 4);
  t.w = w;
  t.h = h;
  t.present = true;
  c->tex_dirty = true;
  return CSG_OK;
}

static LightDev to_light(const csg_light* L) {
  LightDev d;
  for (int k = 0; k < 3; ++k) {
    d.ambient[k] = L->ambient[k];
    d.sun[k] = L->sun[k];
    d.sun_dir[k] = L->sun_dir[k];
  }
  d.sky = (uint32_t)L->sky[0] | ((uint32_t)L->sky[1] << 8) | ((uint32_t)L->sky[2] << 16);
  return d;
}

int csg_set_light(csg_ctx* c, const csg_light* L) {
  if (!c || !L) return CSG_ERR_INVALID;
  c->light = to_light(L);
  c->dr_dirty = true;
  return CSG_OK;
}

int csg_set_dr_light(csg_ctx* c, uint32_t set_id, const csg_light* L) {
  if (!c) return CSG_ERR_INVALID;
  if (!L || set_id >= kMaxSets) return c->fail(CSG_ERR_INVALID, "set_dr_light: need a light and set < %u", kMaxSets);
  if (c->dr_light_valid.size() <= set_id) {
    c->dr_light_valid.resize(set_id + 1, 0);
    c->dr_light.resize(set_id + 1);
  }
  c->dr_light[set_id] = to_light(L);
  c->dr_light_valid[set_id] = 1;
  c->dr_dirty = true;
  return CSG_OK;
}

int csg_set_dr_textures(csg_ctx* c, uint32_t set_id, const int32_t* tex, uint32_t n) {
  if (!c) return CSG_ERR_INVALID;
  if (!c->have_scene) return c->fail(CSG_ERR_INVALID, "set_dr_textures: no scene");
  if (!tex || n != c->n_materials || set_id >= kMaxSets)
    return c->fail(CSG_ERR_INVALID, "set_dr_textures: need %u entries, set < %u", c->n_materials, kMaxSets);
  for (uint32_t m = 0; m < n; ++m)
    if (tex[m] < CSG_KEEP_TEXTURE || tex[m] >= 4096)
      return c->fail(CSG_ERR_INVALID, "set_dr_textures: material %u: bad texture id %d", m, tex[m]);
  const size_t need = ((size_t)set_id + 1) * c->n_materials;
  if (c->dr_tex.size() < need) c->dr_tex.resize(need, CSG_KEEP_TEXTURE);
  memcpy(&c->dr_tex[(size_t)set_id * c->n_materials], tex, n * sizeof(int32_t));
  c->dr_dirty = true;
  return CSG_OK;
}

int csg_set_instance_transforms(csg_ctx* c, uint32_t set_id, const float* model4x4, uint32_t n) {
  if (!c) return CSG_ERR_INVALID;
  if (!c->have_scene) return c->fail(CSG_ERR_INVALID, "set_instance_transforms: no scene");
  if (!model4x4 || n != c->n_inst || set_id >= kMaxSets)
    return c->fail(CSG_ERR_INVALID, "set_instance_transforms: need %u matrices, set < %u", c->n_inst, kMaxSets);
  const size_t per = (size_t)c->n_inst * 16;
  if (c->set_valid.size() <= set_id) {
    c->set_valid.resize(set_id + 1, 0);
    c->h_models.resize(c->set_valid.size() * per, 0.f);
  }
  memcpy(&c->h_models[set_id * per], model4x4, per * sizeof(float));
  c->set_valid[set_id] = 1;
  c->models_dirty = true;
  return CSG_OK;
}

int csg_set_keypoints(csg_ctx* c, uint32_t set_id, const float* pts, uint32_t n) {
  if (!c) return CSG_ERR_INVALID;
  if (!pts || set_id >= kMaxSets || n == 0) return c->fail(CSG_ERR_INVALID, "set_keypoints: bad arguments");
  if (c->n_kp && n != c->n_kp) return c->fail(CSG_ERR_INVALID, "set_keypoints: K must stay %u", c->n_kp);
  c->n_kp = n;
  if (c->kp_valid.size() <= set_id) {
    c->kp_valid.resize(set_id + 1, 0);
    c->h_kp.resize(c->kp_valid.size() * (size_t)n * 3, 0.f);
  }
  memcpy(&c->h_kp[(size_t)set_id * n * 3], pts, (size_t)n * 3 * sizeof(float));
  c->kp_valid[set_id] = 1;
  c->kp_dirty = true;
  return CSG_OK;
}

// Alpha-test class of every alpha quad (2 bits, 16 per word, indexed like the
// alpha-quad image): 0 = all four alphas <= the threshold (the bilinear value
// is too, the test fails whatever the weights), 1 = all four above it (passes),
// 3 = mixed (k_raster loads the quad and filters).  The threshold is that of
// the alpha-tested materials bound to the texture in any transform set; a
// texture used with two thresholds (or none) stays "mixed" everywhere, so the
// class map never changes a result, it only spares most tests the 4-B quad
// load from the much larger quad image.
static int build_alpha_classes(csg_ctx* c, const std::vector<TexDesc>& td, size_t total, bool tex_changed) {
  std::vector<int> thr(c->textures.size(), -1);   // -1 unused, -2 conflicting
  for (const MatDesc& m : c->h_set_mats) {
    if (!m.alpha_test || m.texture < 0 || (size_t)m.texture >= thr.size()) continue;
    int& t = thr[m.texture];
    if (t == -1) t = (int)m.alpha_threshold;
    else if (t != (int)m.alpha_threshold) t = -2;
  }
  if (!tex_changed && c->acls.p && thr == c->acls_thr) return CSG_OK;   // same textures, same thresholds
  c->acls_thr = thr;
  std::vector<uint32_t> cls((total + 15) / 16 + 1, 0xFFFFFFFFu);
  for (size_t k = 0; k < c->textures.size(); ++k) {
    const HostTexture& t = c->textures[k];
    if (!t.present || thr[k] < 0) continue;
    const uint32_t th = (uint32_t)thr[k];
    for (uint32_t y = 0; y < t.h; ++y)
      for (uint32_t x = 0; x < t.w; ++x) {
        const uint32_t x1 = x + 1 == t.w ? 0 : x + 1, y1 = y + 1 == t.h ? 0 : y + 1;
        auto a = [&](uint32_t xx, uint32_t yy) { return (uint32_t)t.rgba[((size_t)yy * t.w + xx) * 4 + 3]; };
        const uint32_t q[4] = {a(x, y), a(x1, y), a(x, y1), a(x1, y1)};
        const uint32_t mn = std::min(std::min(q[0], q[1]), std::min(q[2], q[3]));
        const uint32_t mx = std::max(std::max(q[0], q[1]), std::max(q[2], q[3]));
        const uint32_t cl = mx <= th ? 0u : mn > th ? 1u : 3u;
        const size_t i = (size_t)td[k].offset + (size_t)y * t.w + x;
        cls[i >> 4] = (cls[i >> 4] & ~(3u << (2 * (i & 15)))) | (cl << (2 * (i & 15)));
      }
  }
  HIP_TRY(c, c->acls.alloc(cls.size()));
  HIP_TRY(c, hipMemcpy(c->acls.p, cls.data(), cls.size() * 4, hipMemcpyHostToDevice));
  return CSG_OK;
}

static int sync_scene_state(csg_ctx* c) {
  const uint32_t n_sets = (uint32_t)c->set_valid.size();
  if (c->tex_dirty || c->dr_dirty || c->models_dirty || (c->kp_dirty && c->n_kp) || c->n_table_sets != n_sets) {
    // the device tables are rewritten (and may be reallocated) below: batches
    // in flight still read them
    const int rc = drain(c);
    if (rc) return rc;
  }
  const bool tex_changed = c->tex_dirty;
  const bool iset_dirty = c->tex_dirty || c->dr_dirty || c->n_table_sets != n_sets || !c->iset.p;
  const bool cls_dirty = c->tex_dirty || c->dr_dirty || c->n_table_sets != n_sets || !c->acls.p;
  std::vector<TexDesc> td(c->textures.size());
  size_t total = 0;
  for (size_t k = 0; k < c->textures.size(); ++k) {
    td[k] = TexDesc{(uint32_t)total, c->textures[k].w, c->textures[k].h, 0};
    total += ((size_t)c->textures[k].w * c->textures[k].h + kTexAlign - 1) / kTexAlign * kTexAlign;
  }
  // raster records carry a texture's offset / kTexAlign in 24 bits (Rec::atex)
  if (total / kTexAlign >= 0xFFFFFFu)
    return c->fail(CSG_ERR_LIMIT, "textures hold %zu texels; at most %u", total, 0xFFFFFFu * kTexAlign);
  if (c->tex_dirty) {
    HIP_TRY(c, c->texels.alloc(std::max<size_t>(total * 4, 4)));
    HIP_TRY(c, c->aquad.alloc(std::max<size_t>(total, 1)));
    HIP_TRY(c, c->texd.alloc(std::max<size_t>(td.size(), 1)));
    std::vector<uint32_t> quad;
    for (size_t k = 0; k < c->textures.size(); ++k)
      if (c->textures[k].present) {
        const HostTexture& t = c->textures[k];
        HIP_TRY(c, hipMemcpy(c->texels.p + (size_t)td[k].offset * 4, t.rgba.data(), t.rgba.size(),
                             hipMemcpyHostToDevice));
        // alpha quads: the four alphas of each texel's bilinear footprint (wrapped)
        quad.resize((size_t)t.w * t.h);
        for (uint32_t y = 0; y < t.h; ++y)
          for (uint32_t x = 0; x < t.w; ++x) {
            const uint32_t x1 = x + 1 == t.w ? 0 : x + 1, y1 = y + 1 == t.h ? 0 : y + 1;
            auto a = [&](uint32_t xx, uint32_t yy) { return (uint32_t)t.rgba[((size_t)yy * t.w + xx) * 4 + 3]; };
            quad[(size_t)y * t.w + x] = a(x, y) | (a(x1, y) << 8) | (a(x, y1) << 16) | (a(x1, y1) << 24);
          }
        HIP_TRY(c, hipMemcpy(c->aquad.p + td[k].offset, quad.data(), quad.size() * 4, hipMemcpyHostToDevice));
      }
    if (!td.empty()) HIP_TRY(c, hipMemcpy(c->texd.p, td.data(), td.size() * sizeof(TexDesc), hipMemcpyHostToDevice));
    c->tex_dirty = false;
  }
  // per-set material and light tables (every set that has transforms)
  if (c->dr_dirty || c->n_table_sets != n_sets) {
    std::vector<MatDesc> sm((size_t)n_sets * c->n_materials);
    std::vector<LightDev> sl(n_sets);
    for (uint32_t set = 0; set < n_sets; ++set) {
      sl[set] = (set < c->dr_light_valid.size() && c->dr_light_valid[set]) ? c->dr_light[set] : c->light;
      for (uint32_t m = 0; m < c->n_materials; ++m) {
        MatDesc d = c->h_mats[m];
        const size_t k = (size_t)set * c->n_materials + m;
        if (k < c->dr_tex.size() && c->dr_tex[k] != CSG_KEEP_TEXTURE) d.texture = c->dr_tex[k];
        sm[(size_t)set * c->n_materials + m] = d;
      }
    }
    HIP_TRY(c, c->set_mats.alloc(std::max<size_t>(sm.size(), 1)));
    HIP_TRY(c, c->lights.alloc(std::max<size_t>(sl.size(), 1)));
    c->h_set_mats = sm;
    if (!sm.empty()) HIP_TRY(c, hipMemcpy(c->set_mats.p, sm.data(), sm.size() * sizeof(MatDesc), hipMemcpyHostToDevice));
    if (!sl.empty()) HIP_TRY(c, hipMemcpy(c->lights.p, sl.data(), sl.size() * sizeof(LightDev), hipMemcpyHostToDevice));
    c->n_table_sets = n_sets;
    c->dr_dirty = false;
  }
  if (cls_dirty) {
    const int rc = build_alpha_classes(c, td, total, tex_changed);
    if (rc) return rc;
  }
  for (size_t k = 0; k < c->h_set_mats.size(); ++k) {
    const int t = c->h_set_mats[k].texture;
    if (t >= 0 && ((size_t)t >= c->textures.size() || !c->textures[t].present))
      return c->fail(CSG_ERR_INVALID, "material %u (set %u) references texture %d that was not uploaded",
                     (unsigned)(k % c->n_materials), (unsigned)(k / c->n_materials), t);
  }
  if (iset_dirty) {   // each instance's material per set, texture descriptors inlined
    std::vector<InstSetDev> is((size_t)n_sets * c->n_inst);
    for (uint32_t set = 0; set < n_sets; ++set)
      for (uint32_t i = 0; i < c->n_inst; ++i) {
        const InstDesc& d = c->h_inst[i];
        const MatDesc& m = c->h_set_mats[(size_t)set * c->n_materials + d.material];
        InstSetDev e{};
        e.tex = (m.texture >= 0 && d.has_uv) ? m.texture : -1;
        e.base = (uint32_t)m.base[0] | ((uint32_t)m.base[1] << 8) | ((uint32_t)m.base[2] << 16);
        e.atex = kNoAlpha;
        if (m.alpha_test && m.texture >= 0) {
          const TexDesc& t = td[(size_t)m.texture];
          e.atex = t.offset;
          e.atex_wh = t.width | (t.height << 16);
          e.athr = m.alpha_threshold;
        }
        e.label = d.label;
        e.alpha_uv = (m.alpha_test && d.has_uv) ? 1u : 0u;
        is[(size_t)set * c->n_inst + i] = e;
      }
    HIP_TRY(c, c->iset.alloc(std::max<size_t>(is.size(), 1)));
    if (!is.empty()) HIP_TRY(c, hipMemcpy(c->iset.p, is.data(), is.size() * sizeof(InstSetDev), hipMemcpyHostToDevice));
  }
  if (c->models_dirty) {
    HIP_TRY(c, c->models.alloc(c->h_models.size()));
    HIP_TRY(c, hipMemcpy(c->models.p, c->h_models.data(), c->h_models.size() * 4, hipMemcpyHostToDevice));
    c->models_dirty = false;
  }
  if (c->kp_dirty && c->n_kp) {
    HIP_TRY(c, c->kp.alloc(c->h_kp.size()));
    HIP_TRY(c, hipMemcpy(c->kp.p, c->h_kp.data(), c->h_kp.size() * 4, hipMemcpyHostToDevice));
    c->kp_dirty = false;
  }
  return CSG_OK;
}

// Record cap no frame can exceed: every triangle, plus 1/8 for the second
// triangle of near-plane clips (and slack), rounded to 16-B rect rows.
static uint32_t full_record_cap(const csg_ctx* c) {
  const uint64_t n = std::min<uint64_t>(c->n_tris_total + c->n_tris_total / 8 + 4096, 0x7FFFFFF0ull);
  return (uint32_t)((n + 3u) & ~3ull);
}

// Device bytes ensure_work allocates for a launch chain of F frames with
// pools of the given entries.
static uint64_t work_bytes_for(const csg_ctx* c, uint64_t F, uint64_t rec_pool, uint64_t bin_pool) {
  const uint64_t per_frame = (uint64_t)c->n_tiles * 4 * (2 + c->bin_blocks) + 4 + (uint64_t)c->n_inst * 12 * 4 +
                             12 * 4 + kCamFloats * 4 + kCounterStride * 4 + 4 + sizeof(Slab);
  return rec_pool * (sizeof(Rec) + 4) + bin_pool * 4 + F * per_frame +
         (uint64_t)c->cfg.max_frames * sizeof(FrameDev);
}

static void release_work(csg_ctx* c) {
  c->recs.release(); c->rect.release(); c->bins.release(); c->bcount.release();
  c->tile_count.release(); c->tile_off.release(); c->rec_count.release();
  c->clip.release(); c->pv.release(); c->cam.release(); c->fset.release(); c->slab.release();
  c->work_frames = 0;
  c->rec_pool = c->bin_pool = 0;
  c->last_F = 0;   // the last chain's counters are gone (csg_get_batch_stats: no frames)
}

// Pools a launch chain of F frames gets: sized from the frame hints by
// csg_size_work, else F frames at the per-frame caps.
static void target_pools(const csg_ctx* c, uint32_t F, uint64_t& rp, uint64_t& bp) {
  if (c->use_hints) {
    rp = c->plan_rec_pool;
    bp = c->plan_bin_pool;
  } else {
    rp = (uint64_t)F * c->rec_cap;
    bp = (uint64_t)F * ((c->bin_cap + 3u) & ~3u);
  }
}

static int ensure_work(csg_ctx* c) {
  const uint32_t maxF = c->chain_frames;   // work buffers hold one launch chain
  if (c->rec_cap && c->bin_cap && c->work_frames == maxF) {
    uint64_t rp, bp;
    target_pools(c, maxF, rp, bp);
    if (rp == c->rec_pool && bp == c->bin_pool) return CSG_OK;
  }
  {  // buffers are reallocated below
    const int rc = drain(c);
    if (rc) return rc;
  }
  if (!c->rec_cap) c->rec_cap = c->cfg.records_per_frame ? c->cfg.records_per_frame : full_record_cap(c);
  c->rec_cap = (c->rec_cap + 3u) & ~3u;   // 16-B aligned rect rows per frame (k_count / k_bin load 4 at once)
  if (!c->bin_cap)
    c->bin_cap = c->cfg.bins_per_frame ? c->cfg.bins_per_frame
                                       : (uint32_t)std::min<uint64_t>(3ull * c->rec_cap + 16ull * c->n_tiles,
                                                                      0x7FFFFFFCull);
  uint64_t rp, bp;
  target_pools(c, maxF, rp, bp);
  if (rp != c->rec_pool || bp != c->bin_pool) {   // DevBuf keeps a larger buffer: release to shrink
    c->recs.release(); c->rect.release(); c->bins.release();
  }
  HIP_TRY(c, c->frames.alloc(c->cfg.max_frames));   // the whole batch's frame records
  for (uint32_t k = 0; k < csg_ctx::kStaging; ++k)
    if (!c->h_stage[k])
      HIP_TRY(c, hipHostMalloc(reinterpret_cast<void**>(&c->h_stage[k]), sizeof(FrameDev) * c->cfg.max_frames));
  HIP_TRY(c, c->fset.alloc(maxF));
  HIP_TRY(c, c->clip.alloc((size_t)maxF * c->n_inst * 12));
  HIP_TRY(c, c->pv.alloc((size_t)maxF * 12));
  HIP_TRY(c, c->cam.alloc((size_t)maxF * kCamFloats));
  c->rec_pool = c->bin_pool = 0;
  HIP_TRY(c, c->recs.alloc(rp));
  HIP_TRY(c, c->rect.alloc(rp));
  HIP_TRY(c, c->bins.alloc(bp));
  c->rec_pool = rp;
  c->bin_pool = bp;
  HIP_TRY(c, c->rec_count.alloc((size_t)maxF * kCounterStride));
  HIP_TRY(c, c->tile_count.alloc((size_t)maxF * c->n_tiles));
  HIP_TRY(c, c->tile_off.alloc((size_t)maxF * (c->n_tiles + 1)));
  HIP_TRY(c, c->bcount.alloc((size_t)maxF * c->bin_blocks * c->n_tiles));
  HIP_TRY(c, c->slab.alloc(maxF));
  HIP_TRY(c, c->plan_need.alloc(2));
  c->work_frames = maxF;
  return CSG_OK;
}

static SceneDev scene_dev(const csg_ctx* c) {
  SceneDev s{};
  s.tri_pos = c->tri_pos.p; s.tri_uv = c->tri_uv.p; s.inst = c->inst.p;
  s.texd = c->texd.p; s.texels = c->texels.p; s.aquad = c->aquad.p; s.acls = c->acls.p; s.n_inst = c->n_inst;
  s.W = c->cfg.width; s.H = c->cfg.height;
  s.tiles_x = c->tiles_x; s.tiles_y = c->tiles_y; s.n_tiles = c->n_tiles;
  s.near_clip = c->cfg.near_clip; s.far_clip = c->cfg.far_clip;
  s.inv_near = 1.0f / c->cfg.near_clip; s.inv_far = 1.0f / c->cfg.far_clip;
  s.dbg = c->dbg;
  s.uid_shift = c->uid_shift;
  s.rect_ys = c->tiles_y > 256u ? 1u : 0u;   // tile rectangles of taller frames hold tile-row pairs
  return s;
}

// Page-locked host memory (hipHostMalloc / hipHostRegister): only then is a
// D2H hipMemcpyAsync asynchronous; a pageable destination is staged and blocks.
static bool host_pinned(const void* p) {
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

// Host functions on the copy stream (csg_widen.h): a chain's narrowed ids are
// handed to the widening pool once their copy has landed; the batch's last
// host function waits for all of them, so the copy stream -- and the batch's
// stream, which waits on it -- completes only after the int32 ids are written.
struct WidenChain {
  const void* src;
  uint32_t bytes;
  int32_t* dst;
  size_t n;
  std::shared_ptr<WidenLatch> latch;
};
static void widen_submit_cb(void* p) {
  std::unique_ptr<WidenChain> w(static_cast<WidenChain*>(p));
  WidenPool::get().submit(w->src, w->bytes, w->dst, w->n, w->latch);
}
static void widen_wait_cb(void* p) {
  std::unique_ptr<std::shared_ptr<WidenLatch>> l(static_cast<std::shared_ptr<WidenLatch>*>(p));
  (*l)->wait();
}

// fk: file kinds the batch's images will be encoded to (csg_render_batch):
// images only a file needs are rendered to internal scratch.
static int enqueue_batch(csg_ctx* c, const csg_frame* frames, uint32_t F, int frames_on_device, const csg_outputs* out,
                         hipStream_t st, uint32_t fk = 0) {
  if (!c->have_scene) return c->fail(CSG_ERR_INVALID, "render: no scene uploaded");
  if (!frames || !out || F == 0 || F > c->cfg.max_frames)
    return c->fail(CSG_ERR_INVALID, "render: need 1..%u frames", c->cfg.max_frames);
  // One set of work buffers per context: work queued on another stream must
  // finish before this batch reuses them.
  if (c->last_stream && c->last_stream != st) HIP_TRY(c, hipStreamSynchronize(c->last_stream));
  c->last_stream = st;
  int rc = sync_scene_state(c);
  if (rc) return rc;
  if (out->on_device) {   // k_raster writes 4-pixel groups as vector stores (16-B ids, depth, points; 8-B normals)
    auto mis = [](const void* p, uintptr_t a) { return p && ((uintptr_t)p & (a - 1)) != 0; };
    if (mis(out->instance, 16) || mis(out->depth, 16) || mis(out->points, 16) || mis(out->normals, 8) ||
        mis(out->rgb, 4))
      return c->fail(CSG_ERR_INVALID, "render: device outputs must be aligned (instance, depth, points 16 B; "
                                      "normals 8 B; rgb 4 B)");
  }
  rc = ensure_work(c);
  if (rc) return rc;
  const size_t npx = (size_t)c->cfg.width * c->cfg.height;
  const bool dev = out->on_device != 0;
  const bool want_kp = c->n_kp && (out->keypoints_uv || out->keypoints_vis);
  if (!frames_on_device) {
    for (uint32_t f = 0; f < F; ++f) {
      const uint32_t set = frames[f].xform_set;
      if (set >= c->set_valid.size() || !c->set_valid[set])
        return c->fail(CSG_ERR_INVALID, "frame %u: transform set %u not uploaded", f, set);
      if (want_kp && (set >= c->kp_valid.size() || !c->kp_valid[set]))
        return c->fail(CSG_ERR_INVALID, "frame %u: keypoint set %u not uploaded", f, set);
    }
  }
  BatchDev b{};
  const FrameDev* dframes;
  if (frames_on_device) {
    dframes = reinterpret_cast<const FrameDev*>(frames);
  } else {
    static_assert(sizeof(FrameDev) == sizeof(csg_frame), "frame layout");
    const uint32_t slot = c->stage_next;
    c->stage_next = (slot + 1) % csg_ctx::kStaging;
    if (c->stage_busy[slot]) HIP_TRY(c, hipEventSynchronize(c->stage_ev[slot]));   // its last H2D copy is done
    memcpy(c->h_stage[slot], frames, sizeof(FrameDev) * F);
    HIP_TRY(c, hipMemcpyAsync(c->frames.p, c->h_stage[slot], sizeof(FrameDev) * F, hipMemcpyHostToDevice, st));
    HIP_TRY(c, hipEventRecord(c->stage_ev[slot], st));
    c->stage_busy[slot] = true;
    dframes = c->frames.p;
  }
  b.frames = dframes;
  b.fset = c->fset.p;
  b.n_sets = (uint32_t)c->set_valid.size();    // = sets in the models, materials and lights tables
  b.n_kp_sets = (uint32_t)c->kp_valid.size();
  b.models = c->models.p;
  b.mats = c->set_mats.p;
  b.iset = c->iset.p;
  b.lights = c->lights.p;
  b.n_mat = c->n_materials;
  b.clip = c->clip.p;
  b.pv = c->pv.p;
  b.cam = c->cam.p;
  b.recs = c->recs.p;
  b.rect = c->rect.p;
  b.slab = c->slab.p;
  b.rec_count = c->rec_count.p;
  b.tile_count = c->tile_count.p;
  b.bcount = c->bcount.p;
  b.bin_blocks = c->bin_blocks;
  b.tile_off = c->tile_off.p;
  b.bins = c->bins.p;
  b.overflow = c->overflow.p;
  b.n_labels = out->n_labels;
  b.dbg = c->dbg;
  b.kp = c->kp.p;
  b.n_kp = want_kp ? c->n_kp : 0;
  if (dev) {
    b.rgb = out->rgb;
    b.inst = out->instance;
    b.depth = out->depth;
    b.normals = out->normals;
    b.points = out->points;
    b.stats = out->inst_stats;
    b.covered = out->label_covered;
    b.kp_uv = out->keypoints_uv;
    b.kp_vis = out->keypoints_vis;
  } else {
    if (out->rgb) { HIP_TRY(c, c->o_rgb.alloc(F * npx * 3)); b.rgb = c->o_rgb.p; }
    if (out->instance) { HIP_TRY(c, c->o_inst.alloc(F * npx)); b.inst = c->o_inst.p; }
    if (out->depth) { HIP_TRY(c, c->o_depth.alloc(F * npx)); b.depth = c->o_depth.p; }
    if (out->normals) { HIP_TRY(c, c->o_normals.alloc(F * npx * 3)); b.normals = c->o_normals.p; }
    if (out->points) { HIP_TRY(c, c->o_points.alloc(F * npx * 3)); b.points = c->o_points.p; }
    if (out->inst_stats && out->n_labels) {
      HIP_TRY(c, c->o_stats.alloc((size_t)F * out->n_labels * 5));
      b.stats = c->o_stats.p;
    }
    if (out->label_covered && out->n_labels) {
      HIP_TRY(c, c->o_cov.alloc((size_t)F * out->n_labels));
      b.covered = c->o_cov.p;
    }
  }
  if (!out->inst_stats) b.stats = nullptr;
  if (!out->label_covered || !out->n_labels) b.covered = nullptr;
  // images only a file needs go to internal scratch
  if ((fk & (CSG_FILE_RGB_PNG | CSG_FILE_POINTCLOUD_TXT)) && !b.rgb) {
    HIP_TRY(c, c->o_rgb.alloc(F * npx * 3));
    b.rgb = c->o_rgb.p;
  }
  if ((fk & CSG_FILE_POINTCLOUD_TXT) && !b.points) {
    HIP_TRY(c, c->o_points.alloc(F * npx * 3));
    b.points = c->o_points.p;
  }
  if ((fk & CSG_FILE_DEPTH_CSV || out->depth_stats) && !b.depth) {
    HIP_TRY(c, c->o_depth.alloc(F * npx));
    b.depth = c->o_depth.p;
  }
  // depth visualisation: needs the depth image (internal scratch when the
  // caller did not ask for depth itself)
  const bool want_dvis = out->depth_vis || out->depth_range || (fk & CSG_FILE_DEPTH_PNG);
  uint8_t* dvis = nullptr;
  float* drange_out = nullptr;
  if (want_dvis) {
    if (!b.depth) {
      HIP_TRY(c, c->o_depth.alloc(F * npx));
      b.depth = c->o_depth.p;
    }
    HIP_TRY(c, c->drange.alloc((size_t)2 * c->chain_frames));
    if (out->depth_vis || (fk & CSG_FILE_DEPTH_PNG)) {
      if (dev && out->depth_vis) dvis = out->depth_vis;
      else { HIP_TRY(c, c->o_dvis.alloc(F * npx * 3)); dvis = c->o_dvis.p; }
    }
    if (out->depth_range) {
      if (dev) drange_out = out->depth_range;
      else { HIP_TRY(c, c->o_drange.alloc((size_t)F * 2)); drange_out = c->o_drange.p; }
    }
  }
  double* dstats = nullptr;
  if (out->depth_stats) {
    HIP_TRY(c, c->dstat_part.alloc(depth_stats_scratch_bytes(c->chain_frames)));
    if (dev) dstats = out->depth_stats;
    else { HIP_TRY(c, c->o_dstats.alloc((size_t)F * 6)); dstats = c->o_dstats.p; }
  }
  b.tile_words = (c->n_tiles + 31u) / 32u;
  if (want_kp) {
    HIP_TRY(c, c->kp_w.alloc((size_t)c->chain_frames * c->n_kp));
    HIP_TRY(c, c->kp_pix.alloc((size_t)c->chain_frames * c->n_kp));
    HIP_TRY(c, c->kp_tiles.alloc((size_t)c->chain_frames * b.tile_words));
    b.kp_w = c->kp_w.p;
    b.kp_pix = c->kp_pix.p;
    b.kp_tiles = c->kp_tiles.p;
    if (!b.kp_uv) { HIP_TRY(c, c->o_kp_uv.alloc((size_t)F * c->n_kp * 2)); b.kp_uv = c->o_kp_uv.p; }
    if (!b.kp_vis) { HIP_TRY(c, c->o_kp_vis.alloc((size_t)F * c->n_kp)); b.kp_vis = c->o_kp_vis.p; }
  }
  SceneDev s = scene_dev(c);
  // The batch runs as consecutive launch chains of `chain_frames` frames (by
  // default one chain); the work buffers hold one chain.  With host outputs the
  // chains are at most an eighth of the batch (>= kMinCopyChain frames) and each
  // chain's outputs cross PCIe on the copy stream while the next chains render:
  // the batch then costs about its copies plus one chain's render, not the sum.
  // Pageable destinations are split too: a pageable copy blocks the host until
  // it is done, so later chains do not render under it, but the
  // narrowed ids of each chain are widened on host threads while the next
  // chain's outputs copy, and the copies start before the whole batch is
  // rendered.  Measured (tools/pageable_ab.py, C3 1080p, 480 frames of RGB8 +
  // ids + keypoints into numpy arrays, median of 5): one chain 0.556 s, split
  // 0.509 s (-8.5%); page-locked outputs 0.076 s.  Narrowed ids land in the
  // context's own page-locked buffer, whatever the caller's int32 array is.
  constexpr uint32_t kCopyChunks = 8, kMinCopyChain = 32;
  uint32_t G = c->chain_frames;
  const bool narrow = !dev && out->instance && c->narrow_ids && c->ids_bytes < 4;
  if (!dev) {
    bool pinned = true;
    const void* dsts[] = {out->rgb, narrow ? nullptr : out->instance, out->depth, out->normals, out->points,
                          out->inst_stats, out->label_covered, out->depth_vis, out->depth_range, out->depth_stats,
                          want_kp ? out->keypoints_uv : nullptr, want_kp ? out->keypoints_vis : nullptr};
    for (const void* d : dsts) pinned = pinned && (!d || host_pinned(d));
    if (pinned || c->split_pageable) G = std::min(G, std::max(kMinCopyChain, (F + kCopyChunks - 1) / kCopyChunks));
    if (!c->copy_stream) {
      HIP_TRY(c, hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
      for (auto& e : c->copy_ev) HIP_TRY(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
      HIP_TRY(c, hipEventCreateWithFlags(&c->copy_done, hipEventDisableTiming));
    }
  }
  std::shared_ptr<WidenLatch> latch;
  if (narrow) {
    const size_t nb = (size_t)F * npx * c->ids_bytes;
    HIP_TRY(c, c->o_ids_n.alloc(nb));
    if (c->h_ids_n_bytes < nb) {
      if (c->h_ids_n) {   // the previous batch's widening (on the copy stream) may still read it
        HIP_TRY(c, hipStreamSynchronize(c->copy_stream));
        HIP_TRY(c, hipHostFree(c->h_ids_n));
        c->h_ids_n = nullptr;
        c->h_ids_n_bytes = 0;
      }
      HIP_TRY(c, hipHostMalloc(reinterpret_cast<void**>(&c->h_ids_n), nb, hipHostMallocDefault));
      c->h_ids_n_bytes = nb;
    }
    latch = std::make_shared<WidenLatch>();
  }
  HIP_TRY(c, hipMemsetAsync(c->plan_need.p, 0, 2 * sizeof(uint64_t), st));   // k_plan: max over the chains
  for (uint32_t c0 = 0, chain = 0; c0 < F; c0 += G, ++chain) {
    const uint32_t Fc = std::min(G, F - c0);
    BatchDev bc = b;
    bc.frames = dframes + c0;
    // k_raster's 4-pixel vector stores test the alignment of the absolute pixel
    // index: the chain starts at pixel c0 * npx of the batch's buffers
    bc.px_align = (uint32_t)(((size_t)c0 * npx) & 3u);
    if (bc.rgb) bc.rgb += (size_t)c0 * npx * 3;
    if (bc.inst) bc.inst += (size_t)c0 * npx;
    if (bc.depth) bc.depth += (size_t)c0 * npx;
    if (bc.normals) bc.normals += (size_t)c0 * npx * 3;
    if (bc.points) bc.points += (size_t)c0 * npx * 3;
    if (bc.stats) bc.stats += (size_t)c0 * b.n_labels * 5;
    if (bc.covered) bc.covered += (size_t)c0 * b.n_labels;
    if (want_kp) {
      bc.kp_uv += (size_t)c0 * c->n_kp * 2;
      bc.kp_vis += (size_t)c0 * c->n_kp;
    }
    HIP_TRY(c, hipMemsetAsync(c->rec_count.p, 0, sizeof(uint32_t) * Fc * kCounterStride, st));
    if (want_kp) HIP_TRY(c, hipMemsetAsync(bc.kp_tiles, 0, sizeof(uint32_t) * Fc * bc.tile_words, st));
    launch_init_stats(bc, Fc, st);
    if (bc.covered) HIP_TRY(c, hipMemsetAsync(bc.covered, 0, sizeof(uint32_t) * Fc * b.n_labels, st));
    if (want_dvis) {   // row 0: min (all ones), row 1: max (zero)
      HIP_TRY(c, hipMemsetAsync(c->drange.p, 0xFF, sizeof(uint32_t) * Fc, st));
      HIP_TRY(c, hipMemsetAsync(c->drange.p + Fc, 0, sizeof(uint32_t) * Fc, st));
    }
    bc.drange = want_dvis ? c->drange.p : nullptr;   // reduced by k_raster's resolve
    bc.drange_F = Fc;
    if (c->timing) {
      const uint32_t slot = (uint32_t)(c->ring_count % csg_ctx::kRing);
      c->ev = &c->ring[(size_t)slot * 5];
      c->ring_frames[slot] = Fc;
      ++c->ring_count;
    }
    if (c->timing) HIP_TRY(c, hipEventRecord(c->ev[0], st));
    launch_plan(bc.frames, Fc, c->rec_cap, (c->bin_cap + 3u) & ~3u, c->rec_pool, c->bin_pool, c->use_hints ? 1 : 0,
                c->slab.p, c->plan_need.p, st);
    launch_clip(s, bc, Fc, st);
    launch_setup(s, bc, c->chunks.p, c->n_chunks, Fc, st);
    if (c->timing) HIP_TRY(c, hipEventRecord(c->ev[1], st));
    launch_count(s, bc, Fc, c->bin_blocks, st);
    launch_colscan(s, bc, Fc, st);   // k_count's grid -> block offsets and tile counts
    launch_scan(s, bc, Fc, st);
    launch_bin(s, bc, Fc, c->bin_blocks, st);
    if (c->timing) HIP_TRY(c, hipEventRecord(c->ev[2], st));
    launch_keypoints(s, bc, Fc, st);   // projection; k_raster depth-tests against its z-buffer
    if (c->timing) HIP_TRY(c, hipEventRecord(c->ev[3], st));
    launch_raster(s, bc, Fc, st);
    if (c->timing) HIP_TRY(c, hipEventRecord(c->ev[4], st));
    if (out->depth_stats)
      launch_depth_stats(bc.depth, (uint32_t)npx, Fc, c->dstat_part.p, dstats + (size_t)c0 * 6, st);
    if (want_dvis) {
      if (dvis || drange_out) {
        uint8_t* vo = dvis ? dvis + (size_t)c0 * npx * 3 : nullptr;
        float* ro = drange_out ? drange_out + (size_t)c0 * 2 : nullptr;
        launch_depth_vis(bc.depth, (uint32_t)npx, Fc, c->drange.p, c->jet.p, vo, ro, st);
      }
    }
    c->last_F = Fc;
    if (narrow) launch_narrow_ids(b.inst, (size_t)c0 * npx, (size_t)(c0 + Fc) * npx, c->ids_bytes, c->o_ids_n.p, st);
    if (!dev) {   // this chain's outputs to the host, on the copy stream, behind its kernels
      hipEvent_t e = c->copy_ev[chain % csg_ctx::kCopyEv];
      hipStream_t cs = c->copy_stream;
      HIP_TRY(c, hipEventRecord(e, st));
      HIP_TRY(c, hipStreamWaitEvent(cs, e, 0));
      auto copy = [&](void* dst, const void* src, size_t per_frame) -> hipError_t {
        return hipMemcpyAsync(static_cast<uint8_t*>(dst) + c0 * per_frame,
                              static_cast<const uint8_t*>(src) + c0 * per_frame, Fc * per_frame,
                              hipMemcpyDeviceToHost, cs);
      };
      if (out->rgb) HIP_TRY(c, copy(out->rgb, b.rgb, npx * 3));
      if (narrow) {   // (id + 1) bytes to the landing buffer, then widened into the caller's int32 ids
        const size_t pf = npx * c->ids_bytes;
        HIP_TRY(c, copy(c->h_ids_n, c->o_ids_n.p, pf));
        auto* w = new WidenChain{c->h_ids_n + (size_t)c0 * pf, c->ids_bytes, out->instance + (size_t)c0 * npx,
                                 (size_t)Fc * npx, latch};
        const hipError_t he = hipLaunchHostFunc(cs, widen_submit_cb, w);
        if (he != hipSuccess) delete w;
        HIP_TRY(c, he);
      } else if (out->instance) {
        HIP_TRY(c, copy(out->instance, b.inst, npx * 4));
      }
      if (out->depth) HIP_TRY(c, copy(out->depth, b.depth, npx * 4));
      if (out->normals) HIP_TRY(c, copy(out->normals, b.normals, npx * 6));
      if (out->points) HIP_TRY(c, copy(out->points, b.points, npx * 12));
      if (b.stats) HIP_TRY(c, copy(out->inst_stats, b.stats, (size_t)out->n_labels * 5 * 4));
      if (b.covered) HIP_TRY(c, copy(out->label_covered, b.covered, (size_t)out->n_labels * 4));
      if (out->depth_vis) HIP_TRY(c, copy(out->depth_vis, dvis, npx * 3));
      if (drange_out) HIP_TRY(c, copy(out->depth_range, drange_out, 8));
      if (dstats) HIP_TRY(c, copy(out->depth_stats, dstats, 48));
      if (want_kp && out->keypoints_uv) HIP_TRY(c, copy(out->keypoints_uv, b.kp_uv, (size_t)c->n_kp * 8));
      if (want_kp && out->keypoints_vis) HIP_TRY(c, copy(out->keypoints_vis, b.kp_vis, (size_t)c->n_kp * 4));
    }
  }
  HIP_TRY(c, hipGetLastError());
  c->last_rgb = b.rgb;
  c->last_depth = b.depth;
  c->last_points = b.points;
  c->last_dvis = dvis;
  if (!dev) {   // the batch's stream orders everything after it (and csg_synchronize) behind the copies
    if (narrow) {   // ... and behind the widening of every chain's ids
      auto* l = new std::shared_ptr<WidenLatch>(latch);
      const hipError_t he = hipLaunchHostFunc(c->copy_stream, widen_wait_cb, l);
      if (he != hipSuccess) delete l;
      HIP_TRY(c, he);
    }
    HIP_TRY(c, hipEventRecord(c->copy_done, c->copy_stream));
    HIP_TRY(c, hipStreamWaitEvent(st, c->copy_done, 0));
  }
  return CSG_OK;
}

int csg_render_batch_async(csg_ctx* c, const csg_frame* frames, uint32_t n_frames, int32_t frames_on_device,
                           const csg_outputs* out, void* stream) {
  if (!c) return CSG_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->cfg.device));
  hipStream_t st = stream ? reinterpret_cast<hipStream_t>(stream) : c->stream;
  if (out && out->file_kinds) return c->fail(CSG_ERR_INVALID, "render: file outputs need csg_render_batch");
  return enqueue_batch(c, frames, n_frames, frames_on_device, out, st);
}

int csg_synchronize(csg_ctx* c) {
  if (!c) return CSG_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->cfg.device));
  const int rc = drain(c);
  if (rc) return rc;
  return take_flags(c, nullptr);
}

// Copy the last encoded batch's files to host memory (sizes known).
static int copy_files(csg_ctx* c, uint8_t* dst, uint64_t cap, uint64_t* offsets) {
  if (offsets) memcpy(offsets, c->h_foff.data(), sizeof(uint64_t) * (c->enc_nfiles + 1));
  if (c->enc_total > cap || (!dst && c->enc_total))
    return c->fail(CSG_ERR_CAPACITY, "files: %llu bytes needed, buffer holds %llu",
                   (unsigned long long)c->enc_total, (unsigned long long)cap);
  if (c->enc_total) HIP_TRY(c, hipMemcpyAsync(dst, c->enc_out.p, c->enc_total, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return CSG_OK;
}

// The files of a rendered batch (csg_outputs.file_kinds), encoded on the GPU
// from the images still in HBM (csg_encode.hip): sizes first, then one
// synchronisation to size the buffers, then the bytes, then one D2H copy.
static int encode_files(csg_ctx* c, const csg_outputs* out, uint32_t F) {
  const uint32_t fk = out->file_kinds;
  uint32_t nk = 0, slot_rgb = 0, slot_csv = 0, slot_dpng = 0, slot_pcd = 0;
  if (fk & CSG_FILE_RGB_PNG) slot_rgb = nk++;
  if (fk & CSG_FILE_DEPTH_CSV) slot_csv = nk++;
  if (fk & CSG_FILE_DEPTH_PNG) slot_dpng = nk++;
  if (fk & CSG_FILE_POINTCLOUD_TXT) slot_pcd = nk++;
  const uint32_t W = c->cfg.width, H = c->cfg.height, n_files = F * nk;
  hipStream_t st = c->stream;
  const size_t rows = (size_t)F * png_units_per_frame(W, H), csv_rows = (size_t)F * csv_units_per_frame(W, H);
  HIP_TRY(c, c->enc_fsize.alloc(n_files));
  HIP_TRY(c, c->enc_foff.alloc(n_files + 1));
  HIP_TRY(c, c->enc_zoff.alloc(2 * (size_t)F + 1));
  if (fk & (CSG_FILE_RGB_PNG | CSG_FILE_DEPTH_PNG)) HIP_TRY(c, c->enc_rowsum.alloc(rows));
  if (fk & CSG_FILE_RGB_PNG) {
    HIP_TRY(c, c->enc_rgb.alloc(F));
    HIP_TRY(c, c->enc_rows_rgb.alloc(rows));
    launch_png_sizes(c->last_rgb, W, H, F, c->enc_rgb.p, c->enc_rowsum.p, c->enc_rows_rgb.p, c->enc_fsize.p, nk,
                     slot_rgb, st);
  }
  if (fk & CSG_FILE_DEPTH_PNG) {
    HIP_TRY(c, c->enc_dpng.alloc(F));
    HIP_TRY(c, c->enc_rows_dpng.alloc(rows));
    launch_png_sizes(c->last_dvis, W, H, F, c->enc_dpng.p, c->enc_rowsum.p, c->enc_rows_dpng.p, c->enc_fsize.p, nk,
                     slot_dpng, st);
  }
  if (fk & CSG_FILE_DEPTH_CSV) {
    HIP_TRY(c, c->enc_rows_csv.alloc(csv_rows));
    launch_csv_sizes(c->last_depth, W, H, F, c->enc_rows_csv.p, c->enc_fsize.p, nk, slot_csv, st);
  }
  if (fk & CSG_FILE_POINTCLOUD_TXT) {
    HIP_TRY(c, c->enc_rows_pcd.alloc(csv_rows));
    launch_pcd_sizes(c->last_points, c->last_rgb, W, H, F, c->enc_rows_pcd.p, c->enc_fsize.p, nk, slot_pcd, st);
  }
  const EncPng* pa = (fk & CSG_FILE_RGB_PNG) ? c->enc_rgb.p : nullptr;
  const EncPng* pb = (fk & CSG_FILE_DEPTH_PNG) ? c->enc_dpng.p : nullptr;
  launch_file_layout(c->enc_fsize.p, n_files, c->enc_foff.p, pa, pb, F, c->enc_zoff.p, st);
  HIP_TRY(c, hipGetLastError());
  c->h_foff.resize(n_files + 1);
  uint64_t ztotal = 0;
  HIP_TRY(c, hipMemcpyAsync(c->h_foff.data(), c->enc_foff.p, sizeof(uint64_t) * (n_files + 1), hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipMemcpyAsync(&ztotal, c->enc_zoff.p + 2 * (size_t)F, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipStreamSynchronize(st));
  const uint64_t total = c->h_foff[n_files];
  HIP_TRY(c, c->enc_out.alloc(total + 4));
  if (ztotal) {
    HIP_TRY(c, c->enc_zbuf.alloc(ztotal));
    HIP_TRY(c, hipMemsetAsync(c->enc_zbuf.p, 0, ztotal, st));
  }
  if (pa)
    launch_png_emit(c->last_rgb, W, H, F, pa, c->enc_rows_rgb.p, c->enc_zbuf.p, c->enc_zoff.p, c->enc_out.p,
                    c->enc_foff.p, nk, slot_rgb, st);
  if (pb)
    launch_png_emit(c->last_dvis, W, H, F, pb, c->enc_rows_dpng.p, c->enc_zbuf.p, c->enc_zoff.p + F, c->enc_out.p,
                    c->enc_foff.p, nk, slot_dpng, st);
  if (fk & CSG_FILE_DEPTH_CSV)
    launch_csv_emit(c->last_depth, W, H, F, c->enc_rows_csv.p, c->enc_out.p, c->enc_foff.p, nk, slot_csv, st);
  if (fk & CSG_FILE_POINTCLOUD_TXT)
    launch_pcd_emit(c->last_points, c->last_rgb, W, H, F, c->enc_rows_pcd.p, c->enc_out.p, c->enc_foff.p, nk, slot_pcd,
                    st);
  HIP_TRY(c, hipGetLastError());
  c->enc_total = total;
  c->enc_nfiles = n_files;
  return copy_files(c, out->files, out->files_cap, out->file_offsets);
}

int csg_render_batch(csg_ctx* c, const csg_frame* frames, uint32_t n_frames, const csg_outputs* out) {
  if (!c) return CSG_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->cfg.device));
  // an earlier asynchronous batch that overflowed is reported, not lost
  int rc = csg_synchronize(c);
  if (rc) return rc;
  if (out && (out->file_kinds & ~(CSG_FILE_RGB_PNG | CSG_FILE_DEPTH_CSV | CSG_FILE_DEPTH_PNG | CSG_FILE_POINTCLOUD_TXT)))
    return c->fail(CSG_ERR_INVALID, "render: unknown file kinds %#x", out->file_kinds);
  const uint32_t fk = out ? out->file_kinds : 0u;
  for (int attempt = 0; attempt < 6; ++attempt) {
    rc = enqueue_batch(c, frames, n_frames, 0, out, c->stream, fk);
    if (rc) return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    uint32_t ov = 0;
    HIP_TRY(c, hipMemcpy(&ov, c->overflow.p, 4, hipMemcpyDeviceToHost));
    if (!ov) return fk ? encode_files(c, out, n_frames) : CSG_OK;
    HIP_TRY(c, hipMemsetAsync(c->overflow.p, 0, 4, c->stream));   // before the re-render, on its stream
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (ov & (kOvBadSet | kOvBadKpSet))   // host frames are validated before launch: cannot happen
      return c->fail(CSG_ERR_DEVICE, "render: unexpected set error flags %u", ov);
    // Pools planned from frame hints (csg_size_work) overflowed: another
    // grouping of frames into chains than the sizing assumed (a chain's hints
    // add up past the pool: k_plan's need[]), or stale hints / unmeasured
    // frames (a frame past its own hint).  The first is retried with the pools
    // grown to the largest chain's need, hints kept; the second without hints,
    // every frame at the per-frame caps (the largest measured counts with the
    // margin).  A later csg_size_work turns the hints back on.
    if (c->use_hints) {
      uint64_t need[2] = {0, 0};
      HIP_TRY(c, hipMemcpy(need, c->plan_need.p, sizeof(need), hipMemcpyDeviceToHost));
      if (need[0] > c->rec_pool || need[1] > c->bin_pool) {
        fprintf(stderr, "[csg] hinted work pools too small for this grouping of frames (records %llu > %llu or "
                        "bin entries %llu > %llu): pools grown, re-rendering\n",
                (unsigned long long)need[0], (unsigned long long)c->rec_pool, (unsigned long long)need[1],
                (unsigned long long)c->bin_pool);
        c->plan_rec_pool = std::max<uint64_t>(c->plan_rec_pool, need[0]);
        c->plan_bin_pool = std::max<uint64_t>(c->plan_bin_pool, need[1]);
        ++c->hint_fallbacks;
        continue;
      }
      fprintf(stderr, "[csg] a frame overflowed its work hint (stale hints or an unmeasured frame): hints off, "
                      "re-rendering at the per-frame caps (%u records, %u bin entries per frame); csg_size_work "
                      "turns them back on\n", c->rec_cap, c->bin_cap);
      c->use_hints = false;
      ++c->hint_fallbacks;
      continue;
    }
    // grow the overflowed capacity and re-render (results are a pure function
    // of inputs): at least double it, or size it from the last launch chain's
    // counters (records counted past the cap; bin totals of the records kept)
    uint32_t need_rec = 0, need_bin = 0;
    if (c->last_F) {
      std::vector<uint32_t> cnt((size_t)c->last_F * kCounterStride);
      HIP_TRY(c, hipMemcpy(cnt.data(), c->rec_count.p, cnt.size() * 4, hipMemcpyDeviceToHost));
      std::vector<uint32_t> off((size_t)c->last_F * (c->n_tiles + 1));
      HIP_TRY(c, hipMemcpy(off.data(), c->tile_off.p, off.size() * 4, hipMemcpyDeviceToHost));
      for (uint32_t f = 0; f < c->last_F; ++f) {
        need_rec = std::max(need_rec, cnt[(size_t)f * kCounterStride]);
        need_bin = std::max(need_bin, off[(size_t)f * (c->n_tiles + 1) + c->n_tiles]);
      }
    }
    auto grow = [](uint32_t cap, uint32_t need) {
      return (uint32_t)std::min<uint64_t>(std::max<uint64_t>(2ull * cap, need + need / 8ull + 1024ull), 0x7FFFFFFFull);
    };
    if (ov & kOvRecords) c->rec_cap = (grow(c->rec_cap, need_rec) + 3u) & ~3u;
    if (ov & kOvBins) c->bin_cap = grow(c->bin_cap, need_bin);
    if (ov & kOvRecords) c->bin_cap = grow(c->bin_cap, 0);   // more records: more bin entries too
    c->work_frames = 0;
  }
  return c->fail(CSG_ERR_OVERFLOW, "work buffers overflowed after growth");
}

int csg_copy_files(csg_ctx* c, uint8_t* dst, uint64_t cap, uint64_t* offsets) {
  if (!c) return CSG_ERR_INVALID;
  if (!c->enc_nfiles) return c->fail(CSG_ERR_INVALID, "copy_files: no batch with files rendered");
  HIP_TRY(c, hipSetDevice(c->cfg.device));
  return copy_files(c, dst, cap, offsets);
}

int csg_host_alloc(csg_ctx* c, uint64_t bytes, void** out) {
  if (!c || !out) return CSG_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->cfg.device));
  *out = nullptr;
  HIP_TRY(c, hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault));
  return CSG_OK;
}

int csg_host_free(csg_ctx* c, void* p) {
  if (!c) return CSG_ERR_INVALID;
  if (p) HIP_TRY(c, hipHostFree(p));
  return CSG_OK;
}

int csg_get_batch_stats(csg_ctx* c, csg_batch_stats* st) {
  if (!c || !st) return CSG_ERR_INVALID;
  memset(st, 0, sizeof(*st));
  {
    const int rc = drain(c);
    if (rc) return rc;
  }
  const uint32_t F = c->last_F;
  st->frames = F;
  if (!F) return CSG_OK;
  std::vector<uint32_t> rcs((size_t)F * kCounterStride), rc(F), to((size_t)F * (c->n_tiles + 1));
  std::vector<Slab> sl(F);
  HIP_TRY(c, hipMemcpy(rcs.data(), c->rec_count.p, rcs.size() * 4, hipMemcpyDeviceToHost));
  for (uint32_t f = 0; f < F; ++f) rc[f] = rcs[(size_t)f * kCounterStride];
  HIP_TRY(c, hipMemcpy(to.data(), c->tile_off.p, to.size() * 4, hipMemcpyDeviceToHost));
  HIP_TRY(c, hipMemcpy(sl.data(), c->slab.p, sl.size() * sizeof(Slab), hipMemcpyDeviceToHost));
  for (uint32_t f = 0; f < F; ++f) {
    st->records += std::min(rc[f], sl[f].rec_cap);
    st->bin_entries += to[(size_t)f * (c->n_tiles + 1) + c->n_tiles];
  }
  if (c->timing) {
    float a = 0, b = 0, d = 0, e = 0;
    HIP_TRY(c, hipEventElapsedTime(&a, c->ev[0], c->ev[1]));
    HIP_TRY(c, hipEventElapsedTime(&b, c->ev[1], c->ev[2]));
    HIP_TRY(c, hipEventElapsedTime(&d, c->ev[2], c->ev[3]));
    HIP_TRY(c, hipEventElapsedTime(&e, c->ev[3], c->ev[4]));
    st->ms_setup = a;
    st->ms_bin = b;
    st->ms_keypoints = d;
    st->ms_raster = e;
    st->ms_total = a + b + d + e;
  }
  return CSG_OK;
}

int csg_timing_reset(csg_ctx* c) {
  if (!c) return CSG_ERR_INVALID;
  {
    const int rc = drain(c);
    if (rc) return rc;
  }
  c->ring_count = 0;
  return CSG_OK;
}

int csg_timing_read(csg_ctx* c, csg_timing* out) {
  if (!c || !out) return CSG_ERR_INVALID;
  memset(out, 0, sizeof(*out));
  const uint64_t n = std::min<uint64_t>(c->ring_count, csg_ctx::kRing);
  for (uint64_t k = 0; k < n; ++k) {
    hipEvent_t* e = &c->ring[(size_t)k * 5];
    HIP_TRY(c, hipEventSynchronize(e[4]));
    float a = 0, b = 0, d = 0, f = 0;
    HIP_TRY(c, hipEventElapsedTime(&a, e[0], e[1]));
    HIP_TRY(c, hipEventElapsedTime(&b, e[1], e[2]));
    HIP_TRY(c, hipEventElapsedTime(&d, e[2], e[3]));
    HIP_TRY(c, hipEventElapsedTime(&f, e[3], e[4]));
    out->ms_setup += a;
    out->ms_bin += b;
    out->ms_keypoints += d;
    out->ms_raster += f;
    out->frames += c->ring_frames[k];
  }
  out->batches = (uint32_t)n;
  return CSG_OK;
}

// Sizing pass: k_clip, k_setup, k_count, k_colscan and k_scan over the
// frames in chains of kProbeFrames, with a record cap no frame can exceed
// and no bin cap (k_bin is not run); per frame the record count (k_setup's
// counter, which counts past the cap) and the bin total (tile_off[n_tiles]).
static int measure_work(csg_ctx* c, const csg_frame* frames, uint32_t n, bool on_device, std::vector<uint32_t>& recs_n,
                        std::vector<uint32_t>& bins_n) {
  constexpr uint32_t kProbeFrames = 64;
  const uint32_t P = std::min(kProbeFrames, n);
  uint32_t cap = full_record_cap(c);
  recs_n.assign(n, 0);
  bins_n.assign(n, 0);
  DevBuf<FrameDev> hframes;
  if (!on_device) HIP_TRY(c, hframes.alloc(P));
  SceneDev s = scene_dev(c);
  hipStream_t st = c->stream;
  for (int attempt = 0; attempt < 4; ++attempt) {
    release_work(c);
    HIP_TRY(c, c->fset.alloc(P));
    HIP_TRY(c, c->clip.alloc((size_t)P * c->n_inst * 12));
    HIP_TRY(c, c->pv.alloc((size_t)P * 12));
    HIP_TRY(c, c->cam.alloc((size_t)P * kCamFloats));
    HIP_TRY(c, c->recs.alloc((size_t)P * cap));
    HIP_TRY(c, c->rect.alloc((size_t)P * cap));
    HIP_TRY(c, c->rec_count.alloc((size_t)P * kCounterStride));
    HIP_TRY(c, c->tile_count.alloc((size_t)P * c->n_tiles));
    HIP_TRY(c, c->tile_off.alloc((size_t)P * (c->n_tiles + 1)));
    HIP_TRY(c, c->bcount.alloc((size_t)P * c->bin_blocks * c->n_tiles));
    HIP_TRY(c, c->slab.alloc(P));
    HIP_TRY(c, c->plan_need.alloc(2));
    uint32_t worst = 0;
    for (uint32_t c0 = 0; c0 < n; c0 += P) {
      const uint32_t Fc = std::min(P, n - c0);
      const FrameDev* df;
      if (on_device) {
        df = reinterpret_cast<const FrameDev*>(frames) + c0;
      } else {
        HIP_TRY(c, hipMemcpy(hframes.p, frames + c0, sizeof(FrameDev) * Fc, hipMemcpyHostToDevice));
        df = hframes.p;
      }
      BatchDev b{};
      b.frames = df;
      b.fset = c->fset.p;
      b.n_sets = (uint32_t)c->set_valid.size();
      b.n_kp_sets = (uint32_t)c->kp_valid.size();
      b.models = c->models.p;
      b.mats = c->set_mats.p;
      b.iset = c->iset.p;
      b.lights = c->lights.p;
      b.n_mat = c->n_materials;
      b.clip = c->clip.p;
      b.pv = c->pv.p;
      b.cam = c->cam.p;
      b.recs = c->recs.p;
      b.rect = c->rect.p;
      b.slab = c->slab.p;
      b.rec_count = c->rec_count.p;
      b.tile_count = c->tile_count.p;
      b.bcount = c->bcount.p;
      b.bin_blocks = c->bin_blocks;
      b.tile_off = c->tile_off.p;
      b.overflow = c->overflow.p;
      b.dbg = c->dbg;
      b.tile_words = (c->n_tiles + 31u) / 32u;
      HIP_TRY(c, hipMemsetAsync(c->rec_count.p, 0, sizeof(uint32_t) * Fc * kCounterStride, st));
      // uniform slabs at the probe cap; no bin cap (no bin pool: k_bin is not run)
      launch_plan(df, Fc, cap, 0x7FFFFFFCu, (uint64_t)P * cap, (uint64_t)P * 0x7FFFFFFCull, 0, c->slab.p,
                  c->plan_need.p, st);
      launch_clip(s, b, Fc, st);
      launch_setup(s, b, c->chunks.p, c->n_chunks, Fc, st);
      launch_count(s, b, Fc, c->bin_blocks, st);
      launch_colscan(s, b, Fc, st);
      launch_scan(s, b, Fc, st);
      HIP_TRY(c, hipGetLastError());
      HIP_TRY(c, hipMemcpy2DAsync(recs_n.data() + c0, 4, c->rec_count.p, kCounterStride * 4, 4, Fc,
                                  hipMemcpyDeviceToHost, st));
      HIP_TRY(c, hipMemcpy2DAsync(bins_n.data() + c0, 4, c->tile_off.p + c->n_tiles, (size_t)(c->n_tiles + 1) * 4, 4,
                                  Fc, hipMemcpyDeviceToHost, st));
      HIP_TRY(c, hipStreamSynchronize(st));
      for (uint32_t f = 0; f < Fc; ++f) worst = std::max(worst, recs_n[c0 + f]);
    }
    // k_setup flags records past the cap; device frame records may flag a bad set
    uint32_t ov = 0;
    HIP_TRY(c, hipMemcpy(&ov, c->overflow.p, 4, hipMemcpyDeviceToHost));
    if (ov) {
      HIP_TRY(c, hipMemsetAsync(c->overflow.p, 0, 4, st));
      HIP_TRY(c, hipStreamSynchronize(st));
    }
    if (ov & (kOvBadSet | kOvBadKpSet)) {
      release_work(c);
      return c->fail(CSG_ERR_INVALID, "size_work: device frame records named a transform set >= %u",
                     (unsigned)c->set_valid.size());
    }
    if (worst <= cap) break;   // every frame's records were kept, so its bin total is exact
    if (attempt == 3) {
      release_work(c);
      return c->fail(CSG_ERR_OVERFLOW, "size_work: a frame emitted %u records", worst);
    }
    cap = (uint32_t)std::min<uint64_t>(((uint64_t)worst + worst / 8 + 4096 + 3) & ~3ull, 0x7FFFFFF0ull);
  }
  release_work(c);
  return CSG_OK;
}

static void fill_work_info(const csg_ctx* c, csg_work_info* out) {
  memset(out, 0, sizeof(*out));
  const uint32_t rec = c->rec_cap ? c->rec_cap : (c->cfg.records_per_frame ? c->cfg.records_per_frame : full_record_cap(c));
  const uint32_t bin = c->bin_cap ? c->bin_cap
                                  : (c->cfg.bins_per_frame ? c->cfg.bins_per_frame
                                                           : (uint32_t)std::min<uint64_t>(3ull * rec + 16ull * c->n_tiles,
                                                                                          0x7FFFFFFCull));
  out->records_per_frame = rec;
  out->bins_per_frame = bin;
  out->frames_per_launch = c->chain_frames;
  out->sized_frames = c->sized_frames;
  out->max_records = c->sized_max_rec;
  out->max_bins = c->sized_max_bin;
  out->mean_records = c->sized_mean_rec;
  out->mean_bins = c->sized_mean_bin;
  if (c->use_hints) {
    out->pool_records = c->plan_rec_pool;
    out->pool_bins = c->plan_bin_pool;
  } else {
    out->pool_records = (uint64_t)c->chain_frames * ((rec + 3u) & ~3u);
    out->pool_bins = (uint64_t)c->chain_frames * ((bin + 3u) & ~3u);
  }
  out->hinted = c->use_hints ? 1u : 0u;
  out->hint_retries = c->hint_fallbacks;
  out->work_bytes = work_bytes_for(c, c->chain_frames, out->pool_records, out->pool_bins);
}

// Largest sum of `w` consecutive entries of v (all of v, plus (w - n) x fill,
// when v is shorter than a window).
static uint64_t max_window_sum(const std::vector<uint32_t>& v, uint32_t w, uint32_t fill) {
  const size_t n = v.size();
  if (n <= w) {
    uint64_t t = (uint64_t)(w - n) * fill;
    for (uint32_t x : v) t += x;
    return t;
  }
  uint64_t run = 0, best = 0;
  for (size_t i = 0; i < n; ++i) {
    run += v[i];
    if (i >= w) run -= v[i - w];
    if (i + 1 >= w) best = std::max(best, run);
  }
  return best;
}

int csg_size_work(csg_ctx* c, csg_frame* frames, uint32_t n, int32_t frames_on_device, float margin,
                  csg_work_info* out) {
  if (!c) return CSG_ERR_INVALID;
  if (!frames || n == 0 || !(margin >= 0.0f) || margin > 64.0f)
    return c->fail(CSG_ERR_INVALID, "size_work: need frames and a margin in [0, 64]");
  if (!c->have_scene) return c->fail(CSG_ERR_INVALID, "size_work: no scene uploaded");
  HIP_TRY(c, hipSetDevice(c->cfg.device));
  int rc = csg_synchronize(c);   // earlier batches done (their errors reported), flag clear
  if (rc) return rc;
  if (!frames_on_device)
    for (uint32_t f = 0; f < n; ++f) {
      const uint32_t set = frames[f].xform_set;
      if (set >= c->set_valid.size() || !c->set_valid[set])
        return c->fail(CSG_ERR_INVALID, "size_work: frame %u: transform set %u not uploaded", f, set);
    }
  rc = sync_scene_state(c);
  if (rc) return rc;
  std::vector<uint32_t> rn, bn;
  rc = measure_work(c, frames, n, frames_on_device != 0, rn, bn);
  if (rc) return rc;
  uint32_t mr = 0, mb = 0;
  double sr = 0.0, sb = 0.0;
  for (uint32_t f = 0; f < n; ++f) {
    mr = std::max(mr, rn[f]);
    mb = std::max(mb, bn[f]);
    sr += rn[f];
    sb += bn[f];
  }
  // per-frame caps for unmeasured frames: the largest measured counts
  c->rec_cap = hinted_cap(mr, margin, 256);
  c->bin_cap = hinted_cap(mb, margin, 1024);
  // per-frame hints, written into the frame records: k_plan packs each
  // chain's frames back to back at these sizes
  std::vector<uint32_t> rh(n), bh(n);
  for (uint32_t f = 0; f < n; ++f) {
    rh[f] = hinted_cap(rn[f], margin, 256);
    bh[f] = hinted_cap(bn[f], margin, 1024);
  }
  if (frames_on_device) {
    std::vector<uint32_t> pairs((size_t)2 * n);
    for (uint32_t f = 0; f < n; ++f) { pairs[2 * f] = rh[f]; pairs[2 * f + 1] = bh[f]; }
    HIP_TRY(c, hipMemcpy2DAsync(reinterpret_cast<uint8_t*>(frames) + offsetof(csg_frame, records_hint),
                                sizeof(csg_frame), pairs.data(), 8, 8, n, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
  } else {
    for (uint32_t f = 0; f < n; ++f) {
      frames[f].records_hint = rh[f];
      frames[f].bins_hint = bh[f];
    }
  }
  // pools: the heaviest run of chain_frames consecutive frames of this order
  c->plan_rec_pool = max_window_sum(rh, c->chain_frames, c->rec_cap);
  c->plan_bin_pool = max_window_sum(bh, c->chain_frames, (c->bin_cap + 3u) & ~3u);
  c->use_hints = true;
  c->sized_frames = n;
  c->sized_max_rec = mr;
  c->sized_max_bin = mb;
  c->sized_mean_rec = sr / n;
  c->sized_mean_bin = sb / n;
  release_work(c);   // the next batch allocates the pools at these sizes
  if (out) fill_work_info(c, out);
  return CSG_OK;
}

int csg_get_work_info(csg_ctx* c, csg_work_info* out) {
  if (!c || !out) return CSG_ERR_INVALID;
  fill_work_info(c, out);
  return CSG_OK;
}

int csg_host_id_bytes(const csg_ctx* c) {
  if (!c) return CSG_ERR_INVALID;
  return c->narrow_ids ? (int)c->ids_bytes : 4;
}

int csg_project_keypoints(csg_ctx* c, const float* pts, uint32_t n, const float* view, const float* proj, float* uv_out,
                          int32_t* vis_out) {
  if (!c) return CSG_ERR_INVALID;
  if (!pts || !view || !proj || !uv_out || !vis_out || n == 0)
    return c->fail(CSG_ERR_INVALID, "project_keypoints: bad arguments");
  HIP_TRY(c, hipSetDevice(c->cfg.device));
  // P*V rows 0,1,3 with the spec's fp32 summation order (host side; 48 products)
  float pv[16];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) {
      volatile float t0 = proj[i * 4 + 0] * view[0 * 4 + j];
      volatile float t1 = proj[i * 4 + 1] * view[1 * 4 + j];
      volatile float s01 = t0 + t1;
      volatile float t2 = proj[i * 4 + 2] * view[2 * 4 + j];
      volatile float s012 = s01 + t2;
      volatile float t3 = proj[i * 4 + 3] * view[3 * 4 + j];
      pv[i * 4 + j] = s012 + t3;
    }
  float pv12[12];
  for (int k = 0; k < 4; ++k) { pv12[k] = pv[k]; pv12[4 + k] = pv[4 + k]; pv12[8 + k] = pv[12 + k]; }
  DevBuf<float> dp, dpv, duv;
  DevBuf<int32_t> dvis;
  HIP_TRY(c, dp.alloc((size_t)n * 3));
  HIP_TRY(c, dpv.alloc(12));
  HIP_TRY(c, duv.alloc((size_t)n * 2));
  HIP_TRY(c, dvis.alloc(n));
  HIP_TRY(c, hipMemcpy(dp.p, pts, (size_t)n * 12, hipMemcpyHostToDevice));
  HIP_TRY(c, hipMemcpy(dpv.p, pv12, 48, hipMemcpyHostToDevice));
  launch_project(dp.p, n, dpv.p, (float)c->cfg.width, (float)c->cfg.height, c->cfg.near_clip, duv.p, dvis.p,
                 c->stream);
  HIP_TRY(c, hipGetLastError());
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  HIP_TRY(c, hipMemcpy(uv_out, duv.p, (size_t)n * 8, hipMemcpyDeviceToHost));
  HIP_TRY(c, hipMemcpy(vis_out, dvis.p, (size_t)n * 4, hipMemcpyDeviceToHost));
  dp.release(); dpv.release(); duv.release(); dvis.release();
  return CSG_OK;
}

int csg_instance_bounds(csg_ctx* c, uint32_t set_id, float* out) {
  if (!c) return CSG_ERR_INVALID;
  if (!out) return c->fail(CSG_ERR_INVALID, "instance_bounds: null output");
  if (set_id >= c->set_valid.size() || !c->set_valid[set_id])
    return c->fail(CSG_ERR_INVALID, "instance_bounds: transform set %u not uploaded", set_id);
  HIP_TRY(c, hipSetDevice(c->cfg.device));
  const int rc = sync_scene_state(c);
  if (rc) return rc;
  const size_t n = (size_t)c->n_inst * 6;
  // ordered-uint encoding: min slots start at max, max slots at 0
  std::vector<uint32_t> init(n);
  for (size_t k = 0; k < n; ++k) init[k] = (k % 6) < 3 ? 0xFFFFFFFFu : 0u;
  DevBuf<uint32_t> d;
  HIP_TRY(c, d.alloc(n));
  HIP_TRY(c, hipMemcpy(d.p, init.data(), n * 4, hipMemcpyHostToDevice));
  launch_inst_bounds(scene_dev(c), c->chunks.p, c->n_chunks, c->models.p + (size_t)set_id * c->n_inst * 16, d.p,
                     c->stream);
  HIP_TRY(c, hipGetLastError());
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  HIP_TRY(c, hipMemcpy(init.data(), d.p, n * 4, hipMemcpyDeviceToHost));
  d.release();
  for (size_t k = 0; k < n; ++k) {
    const uint32_t o = init[k];
    const uint32_t u = (o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o;
    memcpy(&out[k], &u, 4);
  }
  return CSG_OK;
}

}  // extern "C"
