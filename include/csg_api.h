/*
 * csg_api.h — C ABI of the MI355X construction-scene frame generator
 * (libcsg.so, built for gfx950).  Plain C99: no C++ or torch types cross
 * this boundary.  Every entry point returns 0 on success, a negative
 * csg_status on failure; csg_last_error() gives the message.
 *
 * What each entry point replaces in the reference
 * (xander683/ConstructionScenePoseEstimation, generate_construction_data.py):
 *
 *   csg_create ................ Camera(prim_path, resolution) + clip/focal/aperture
 *                               setup + camera.initialize()           :1421-1453
 *   csg_upload_scene .......... the USD stage the RTX renderer reads  :1370
 *   csg_upload_texture ........ material texture binding (OmniPBR
 *                               diffuse/opacity maps)                 world2 materials
 *   csg_set_light ............. setup_scene_lighting (dome 500,
 *                               distant light clamped to 1500)        :1289-1345
 *   csg_set_instance_transforms randomize_object_positions' xformOp
 *                               edits (every 10 frames)               :914-1231, :1542
 *   csg_set_dr_light / ........ per-epoch domain randomisation (dome tint,
 *   csg_set_dr_textures         sun, texture swap; C4 of BASELINE.json)
 *   csg_set_keypoints ......... (new) 3D points whose 2D projection is
 *                               annotated; the reference produces none
 *   csg_render_batch .......... camera.set_world_pose + next_update_async
 *                               + get_rgba / distance_to_image_plane /
 *                               instance_segmentation .get_data()     :1586-1595, :1669,
 *                                                                     :1681, :1475/:1909
 *   csg_project_keypoints ..... 3D->2D projection with the frame's
 *                               intrinsics (pinhole of :646-649)
 *   csg_outputs.file_kinds .... the frame's files encoded on the GPU:
 *                               cv2.imwrite of the RGB and JET depth
 *                               images, np.savetxt of the depth  :1672-1673,
 *                               and of the point cloud           :1687-1709,
 *                                                                :714-775, :1716-1757
 *   csg_copy_files / csg_host_alloc / csg_host_free (pinned buffers for them)
 *   csg_size_work / csg_get_work_info (per-frame work-buffer caps measured
 *                               on a sample of frames; no reference counterpart:
 *                               Kit sizes its own render buffers)
 *   csg_host_id_bytes ......... width of the instance ids on the host wire
 *                               (int32 mask of :1909-1910 narrowed to
 *                               id + 1 bytes on PCIe, widened on the host)
 *   csg_last_error / csg_destroy
 *
 * Threading: several contexts may share a device (each has its own stream
 * and work buffers; the generator drives two from two threads); a context is
 * used by one thread at a time.  The only process-wide state is the pool of
 * host threads that widens narrowed instance ids (csg_host_id_bytes).
 */
#ifndef CSG_API_H
#define CSG_API_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CSG_ABI_VERSION 11

typedef enum {
  CSG_OK = 0,
  CSG_ERR_INVALID = -1,      /* bad argument / state */
  CSG_ERR_DEVICE = -2,       /* HIP runtime error */
  CSG_ERR_OOM = -3,          /* device allocation failed */
  CSG_ERR_OVERFLOW = -4,     /* a per-frame work buffer overflowed; raise caps */
  CSG_ERR_LIMIT = -5,        /* scene exceeds a fixed limit (instances, tris/mesh) */
  CSG_ERR_CAPACITY = -6      /* csg_outputs.files too small: file_offsets[n_files] holds the
                                bytes needed; csg_copy_files fetches them without rendering again */
} csg_status;

typedef struct csg_ctx csg_ctx;

typedef struct {
  int32_t device;            /* HIP device ordinal (after HIP_VISIBLE_DEVICES) */
  uint32_t width, height;    /* output resolution, e.g. 1920x1080; at most 8192 x 8192 (256 x 512
                                tiles of 32 x 16: CSG_ERR_INVALID beyond) */
  uint32_t max_frames;       /* frames per csg_render_batch call (work buffers sized for it) */
  float near_clip, far_clip; /* 0.5 / 250 m, generate_construction_data.py:1437; in [2^-126, 2^126] */
  uint32_t records_per_frame;/* raster-triangle capacity per frame (0 = auto) */
  uint32_t bins_per_frame;   /* tile-bin entry capacity per frame (0 = auto) */
  uint32_t frames_per_launch;/* frames per kernel chain inside a batch (0 = the whole batch):
                                work buffers are sized for one chain, so this bounds their
                                memory independently of max_frames */
} csg_config;

typedef struct {
  const float* positions;    /* [n_vertices][3] object space */
  uint32_t n_vertices;
  const uint32_t* indices;   /* [n_tris][3] */
  uint32_t n_tris;           /* < 2^20 */
  const float* uvs;          /* [n_uvs][2] USD st, or NULL */
  uint32_t n_uvs;
  const uint32_t* uv_indices;/* [n_tris][3] into uvs, or NULL */
  uint32_t material;
} csg_mesh;

typedef struct {
  uint8_t base_color[4];     /* sRGB u8 albedo multiplier (alpha unused) */
  int32_t texture;           /* texture id or -1 */
  uint32_t alpha_test;       /* 1: discard fragments with texture alpha <= threshold */
  uint32_t alpha_threshold;  /* 0..255 (alpha is 8-bit) */
} csg_material;

typedef struct {
  float model[16];           /* row-major 4x4, column-vector convention p' = M p */
  uint32_t mesh;
  int32_t inst_idx;          /* value written to the instance mask; -1 = background */
  uint32_t reserved[2];
} csg_instance;

typedef struct {
  float ambient[3];          /* dome light contribution per channel */
  float sun[3];              /* distant light contribution per channel */
  float sun_dir[3];          /* unit vector toward the sun, world space */
  uint8_t sky[4];            /* background RGB */
} csg_light;

typedef struct {
  float view[16];            /* row-major world->camera (USD camera: -Z forward) */
  float proj[16];            /* row-major; rows 0,1,3 give (u*w, v*w, w) in pixels */
  uint32_t xform_set;        /* instance-transform set (randomisation epoch) */
  uint32_t frame_id;
  uint32_t records_hint;     /* work to reserve for this frame: raster records and tile-bin */
  uint32_t bins_hint;        /* entries; csg_size_work writes them (0 = the per-frame caps) */
} csg_frame;

typedef struct {
  /* Caller-owned buffers, [n_frames] leading dimension.  Any may be NULL. */
  uint8_t* rgb;              /* [n][H][W][3] */
  int32_t* instance;         /* [n][H][W], -1 background */
  float* depth;              /* [n][H][W] distance to image plane, +inf no hit */
  float* keypoints_uv;       /* [n][K][2] pixels */
  int32_t* keypoints_vis;    /* [n][K] 0 out/behind, 1 occluded, 2 visible */
  uint32_t* inst_stats;      /* [n][n_labels][5] = pixels, minx, miny, maxx, maxy */
  uint32_t n_labels;
  int32_t on_device;         /* 1: device pointers (stay in HBM; instance, depth and points
                                16-B aligned, normals 8 B, rgb 4 B: CSG_ERR_INVALID otherwise,
                                as k_raster stores 4-pixel groups), 0: host pointers */
  uint16_t* normals;         /* [n][H][W][3] f16 bits: unit world-space face normal facing
                                the camera; 0 where nothing is hit (C5 normals) */
  float* points;             /* [n][H][W][3] world-space point of each pixel from its depth
                                (depth_to_pointcloud GDP:616-711, fused); NaN where no hit */
  uint8_t* depth_vis;        /* [n][H][W][3] RGB: the reference's depth PNG (GDP:1690-1709):
                                valid depth (finite, > 0) normalised by the frame's min / max,
                                JET colour map (OpenCV COLORMAP_JET), black if nothing is hit */
  float* depth_range;        /* [n][2] min, max of the valid depth (NaN, NaN: nothing hit) */
  uint32_t* label_covered;   /* [n][n_labels] pixels each label would cover unoccluded: a
                                fragment of it covers the centre, lies in the depth range and
                                passes the alpha test (no depth test).  Bit 31 set = unknown
                                (a 32x32 tile held more than 32 labels).  occlusionRatio =
                                1 - pixels / covered (bounding_box_3d, GDP:1780-1790) */
  /* Files encoded on the GPU (csg_render_batch only, not the async form).
   * file_kinds: bit set of CSG_FILE_*; per frame one file per kind, in bit
   * order: file j = frame * n_kinds + k.  The packed bytes of all files go to
   * `files` (host memory, files_cap bytes; pinned memory from csg_host_alloc
   * copies at full PCIe rate), file j at [file_offsets[j], file_offsets[j + 1])
   * (file_offsets: n_frames * n_kinds + 1 entries).  The images a kind needs
   * are rendered to internal scratch when the caller did not ask for them. */
  uint32_t file_kinds;
  uint32_t pad_files;
  uint8_t* files;
  uint64_t files_cap;
  uint64_t* file_offsets;
  double* depth_stats;       /* [n][6] per frame: valid pixels (finite, > 0), zero pixels, infinite
                                pixels, sum / min / max of the valid depths (the reference's
                                DataQualityLogger.log_depth, GDP:318-341); the sum in float64 in a
                                fixed order (64 partial sums per frame, then in order) */
} csg_outputs;

/* csg_outputs.file_kinds */
#define CSG_FILE_RGB_PNG 1u        /* 8-bit RGB PNG of the frame (cv2.imwrite, GDP:1672-1673): filter Sub,
                                      one dynamic-Huffman deflate block of literals and distance-1 matches,
                                      2 KiB IDAT chunks */
#define CSG_FILE_DEPTH_CSV 2u      /* np.savetxt(depth, fmt="%.6f", delimiter=" ") text (GDP:1687-1688),
                                      byte-identical */
#define CSG_FILE_DEPTH_PNG 4u      /* the JET depth visualisation (csg_outputs.depth_vis) as a PNG
                                      (GDP:1690-1709) */
#define CSG_FILE_POINTCLOUD_TXT 8u /* np.savetxt(np.hstack([xyz, rgb]), fmt="%.6f", delimiter=" ",
                                      header="x y z r g b", comments="") of the pixels with a point
                                      (csg_outputs.points not NaN), row-major (GDP:766-770,
                                      :1716-1757), byte-identical */

typedef struct {
  uint64_t records;          /* raster triangles emitted (all frames of the last launch chain) */
  uint64_t bin_entries;      /* tile-bin entries (same frames) */
  uint32_t frames;           /* frames of the last launch chain */
  uint32_t pad;
  float ms_setup, ms_bin, ms_raster, ms_keypoints, ms_total;   /* HIP-event timings */
} csg_batch_stats;

int csg_create(const csg_config* cfg, csg_ctx** out);
void csg_destroy(csg_ctx* ctx);
const char* csg_last_error(const csg_ctx* ctx);
int csg_abi_version(void);

int csg_upload_scene(csg_ctx* ctx, const csg_mesh* meshes, uint32_t n_meshes,
                     const csg_material* materials, uint32_t n_materials,
                     const csg_instance* instances, uint32_t n_instances);
int csg_upload_texture(csg_ctx* ctx, uint32_t tex_id, const uint8_t* rgba8, uint32_t width,
                       uint32_t height);
int csg_set_light(csg_ctx* ctx, const csg_light* light);
/* n must equal the scene's instance count; set_id < 65536 (also for the per-set calls below). */
int csg_set_instance_transforms(csg_ctx* ctx, uint32_t set_id, const float* model4x4, uint32_t n);
/* World-space keypoints of one transform set: [n][3]; n is fixed per scene. */
int csg_set_keypoints(csg_ctx* ctx, uint32_t set_id, const float* pts_world, uint32_t n);

/* Domain randomisation per transform set (randomisation epoch; C4).
 * csg_set_dr_light: the set's lighting (dome tint/intensity, sun), replacing
 * the csg_set_light default for frames of that set.
 * csg_set_dr_textures: per material, the texture the set uses: a texture id,
 * -1 for none, or CSG_KEEP_TEXTURE for the material's own; n = n_materials. */
#define CSG_KEEP_TEXTURE (-2)
int csg_set_dr_light(csg_ctx* ctx, uint32_t set_id, const csg_light* light);
int csg_set_dr_textures(csg_ctx* ctx, uint32_t set_id, const int32_t* texture_per_material, uint32_t n);

/* Render n_frames (<= max_frames) frames; synchronous.  A work buffer that
 * overflows (records or bin entries past the configured caps) is grown from
 * the device counters and the batch rendered again, up to 6 attempts; the
 * results do not depend on the caps.  An overflow left by an earlier
 * asynchronous batch is reported first (CSG_ERR_OVERFLOW), as by
 * csg_synchronize.  With host outputs the batch runs as launch chains of an
 * eighth of it (at least 32 frames), each chain's outputs copied to the host
 * on a copy stream while later chains render (CSG_SPLIT_PAGEABLE=0 at
 * csg_create: pageable destinations as one chain). */
int csg_render_batch(csg_ctx* ctx, const csg_frame* frames, uint32_t n_frames, const csg_outputs* out);
/* Same, enqueued on `stream` (a hipStream_t, NULL = context stream); frames
 * may be a device pointer when frames_on_device = 1.  Returns after enqueue;
 * the work buffers are not grown.  Host frame records are staged through a
 * ring of pinned buffers, so the caller may reuse `frames` at once.  A batch
 * on a different stream than the previous one waits for that stream first
 * (one set of work buffers per context).  Device frame records are checked on
 * the device: a transform set >= the sets uploaded renders with set 0, a
 * keypoint set never uploaded projects nothing, and both are reported by the
 * next csg_synchronize (CSG_ERR_INVALID).  Sets inside the range that were
 * never uploaded hold zero transforms (nothing is drawn). */
int csg_render_batch_async(csg_ctx* ctx, const csg_frame* frames, uint32_t n_frames,
                           int32_t frames_on_device, const csg_outputs* out, void* stream);
/* Wait for every batch enqueued so far (context stream and the caller's
 * stream of the last batch).  Overflow and device-set errors are sticky
 * across asynchronous batches: any batch since the last csg_synchronize /
 * csg_render_batch that truncated its records or bin lists makes this return
 * CSG_ERR_OVERFLOW (then the flag is cleared). */
int csg_synchronize(csg_ctx* ctx);
int csg_get_batch_stats(csg_ctx* ctx, csg_batch_stats* st);

/* Per-stage device time accumulated with HIP events recorded on the launch
 * stream for every launch chain since the last reset (no host sync inside
 * the timed loop); `batches` counts launch chains.  Stages: setup = k_clip+k_setup, bin = k_count+k_scan+k_bin,
 * keypoints = k_keypoints (projection), raster = k_raster (tile raster,
 * keypoint depth test, resolve). */
typedef struct {
  uint32_t batches;          /* launch chains accumulated (capped at the ring size, 4096) */
  uint32_t frames;           /* frames in those batches */
  double ms_setup, ms_bin, ms_raster, ms_keypoints;
} csg_timing;
int csg_timing_reset(csg_ctx* ctx);
int csg_timing_read(csg_ctx* ctx, csg_timing* out);

/* World-space AABB of each instance's vertices under transform set set_id,
 * out [n_instances][6] = xmin, ymin, zmin, xmax, ymax, zmax (host buffer);
 * the GPU side of the bounding_box_3d annotator (GDP:1780-1790). */
int csg_instance_bounds(csg_ctx* ctx, uint32_t set_id, float* out);

/* The files of the last csg_render_batch that asked for files, again
 * (after CSG_ERR_CAPACITY): dst host memory of cap bytes; offsets as
 * csg_outputs.file_offsets (may be NULL). */
int csg_copy_files(csg_ctx* ctx, uint8_t* dst, uint64_t cap, uint64_t* offsets);
/* Page-locked host memory for csg_outputs.files and the other host outputs. */
int csg_host_alloc(csg_ctx* ctx, uint64_t bytes, void** out);
int csg_host_free(csg_ctx* ctx, void* p);

/* Work-buffer sizing.  k_setup appends each frame's raster records into the
 * frame's region of a record pool and k_bin its tile lists into a region of a
 * bin pool; the pools hold one launch chain (frames_per_launch frames), whose
 * frames get back-to-back regions (a planning kernel at the head of the
 * chain).  A frame's region is its csg_frame hints, or with hints 0 the
 * per-frame caps.  With the config's caps 0 and no sizing those are sized for
 * every triangle of the scene (1.125 x triangles per frame, 3x that in bin
 * entries), which no frame can overflow but which a typical view uses a
 * fraction of (C3 1080p: ~1/5 of the records, ~1/9 of the bin entries).
 *
 * csg_size_work runs the sizing pass on `n_frames` frames (host records, or
 * device records when frames_on_device = 1; any number, in chains of 64):
 * k_clip, k_setup, k_count, k_colscan and k_scan only, no raster and no
 * outputs.  It then
 *   - writes each frame's hints: its measured record and bin-entry counts
 *     times (1 + margin) (margin >= 0, e.g. 0.25) plus a small pad, into
 *     the frame records passed (device or host memory);
 *   - sets the per-frame caps (frames without hints) to the largest counts
 *     measured, with the same margin;
 *   - sizes the pools for the heaviest run of frames_per_launch consecutive
 *     frames of the order given (fewer frames than that: all of them plus
 *     the rest at the per-frame caps),
 * and frees the work buffers (the next batch allocates them).  The counts are
 * a pure function of the frame and the scene, so batches that render the
 * measured frames, in that order, with their hints, never overflow.  Other
 * batches can: csg_render_batch then renders again -- with the pools grown to
 * the largest launch chain's hinted total when the frames were grouped
 * differently, else without hints (every frame at the per-frame caps), then
 * with grown caps -- and prints a "[csg]" line on stderr for each such retry;
 * an asynchronous batch reports CSG_ERR_OVERFLOW at the next csg_synchronize.  Waits for the context's
 * earlier batches first (and reports their errors). */
typedef struct {
  uint32_t records_per_frame;  /* current per-frame caps (frames without hints) */
  uint32_t bins_per_frame;
  uint32_t frames_per_launch;  /* frames the work buffers hold (one launch chain) */
  uint32_t sized_frames;       /* frames the last csg_size_work measured (0: none) */
  uint32_t max_records;        /* largest per-frame counts it measured */
  uint32_t max_bins;
  double mean_records;         /* and their means */
  double mean_bins;
  uint64_t work_bytes;         /* device bytes of the work buffers at the current pools */
  uint64_t pool_records;       /* pool entries of one launch chain */
  uint64_t pool_bins;
  uint32_t hinted;             /* 1: pools sized from frame hints (csg_size_work) */
  uint32_t hint_retries;       /* re-renders the hinted pools caused (grown pools or hints turned off) */
} csg_work_info;
int csg_size_work(csg_ctx* ctx, csg_frame* frames, uint32_t n_frames, int32_t frames_on_device,
                  float margin, csg_work_info* out);
int csg_get_work_info(csg_ctx* ctx, csg_work_info* out);

/* Bytes per instance id on the host wire of host-output batches: 1 when every
 * instance label is in [-1, 254], 2 up to 65,534, else 4 (int32 as rendered).
 * The ids cross PCIe as (id + 1) in that width and are widened into the
 * caller's int32 array on host threads (the reference's int32 mask,
 * generate_construction_data.py:1909-1910, :2066-2069) before the batch's
 * stream completes; CSG_NARROW_IDS=0 at csg_create keeps int32 on the wire.
 * Returns the width (1, 2 or 4), or a negative status. */
int csg_host_id_bytes(const csg_ctx* ctx);

/* Stand-alone 3D->2D projection (host buffers): uv [n][2], vis [n] without a
 * depth test (1 = in front and inside the image, 0 otherwise). */
int csg_project_keypoints(csg_ctx* ctx, const float* pts_world, uint32_t n, const float* view,
                          const float* proj, float* uv_out, int32_t* vis_out);

#ifdef __cplusplus
}
#endif
#endif /* CSG_API_H */
