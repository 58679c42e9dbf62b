/*
 * CPU ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Scalar C restatement of the render + annotate step that the reference
 * obtains from Isaac Sim's closed RTX renderer and Replicator annotators
 * (generate_construction_data.py:1592-1595 render, :1669 get_rgba,
 * :1681 distance_to_image_plane, :1909-1910 instance mask, :1780/:1916
 * bounding_box_3d).  The renderer itself is closed and absent, so render
 * parity is UNPINNED against RTX: this oracle fixes the arithmetic of the
 * path (DESIGN.md "Raster spec") and the GPU kernels must match it
 * bit-for-bit.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it, and only as the checker.
 */
#ifndef CSG_ORACLE_H
#define CSG_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  uint32_t vbase, tbase, ntris, uvbase, has_uv, material;
} oracle_mesh;

typedef struct {
  uint8_t base[4];          /* albedo multiplier, u8 */
  int32_t texture;          /* -1: none */
  uint32_t alpha_test;
  uint32_t alpha_threshold; /* keep iff alpha8 > threshold */
} oracle_material;

typedef struct {
  uint32_t offset;          /* texel offset into the RGBA8 blob */
  uint32_t width, height, pad;
} oracle_texture;

typedef struct {
  /* geometry (global arrays; tris/uv_tris are mesh-relative) */
  const float* positions;       /* [V][3] */
  const uint32_t* tris;         /* [T][3] */
  const float* uvs;             /* [U][2] */
  const uint32_t* uv_tris;      /* [T][3] */
  const oracle_mesh* meshes;
  uint32_t n_meshes;
  /* instances */
  const float* inst_model;      /* [I][16] row-major, p' = M p */
  const uint32_t* inst_mesh;    /* [I] */
  const int32_t* inst_label;    /* [I] inst_idx, -1 background */
  const uint32_t* inst_tri_base;/* [I+1] prefix of triangle counts (uid space) */
  uint32_t n_inst;
  /* materials / textures */
  const oracle_material* materials;
  uint32_t n_materials;
  const uint8_t* texels;        /* RGBA8 blob */
  const oracle_texture* textures;
  uint32_t n_textures;
  /* lighting (float32 constants fixed on the host) */
  float ambient[3], sun[3], sun_dir[3];
  uint8_t sky[4];
  /* camera */
  uint32_t width, height;
  float near_clip, far_clip;
} oracle_scene;

typedef struct {
  uint64_t n_tris_in, n_culled, n_clipped, n_raster_tris, n_fragments, n_alpha_killed;
  uint64_t n_bbox_pixels, n_covered, n_early_z_killed, n_alpha_tests;
} oracle_stats;

/* Render one frame. view/proj: 16 floats row-major (proj rows 0,1,3 used).
 * Outputs may be NULL.  inst_stats: [n_labels][5] = count, minx, miny, maxx, maxy. */
int oracle_render_frame(const oracle_scene* s, const float* view, const float* proj,
                        uint8_t* rgb, int32_t* inst, float* depth,
                        uint32_t* inst_stats, uint32_t n_labels, oracle_stats* st);

/* Same plus the C5 outputs: normals [H][W][3] f16 bits (unit world-space face
 * normal facing the camera, 0 for background) and points [H][W][3] (world
 * point of each pixel from its depth, NaN for background). */
int oracle_render_frame_ex(const oracle_scene* s, const float* view, const float* proj,
                           uint8_t* rgb, int32_t* inst, float* depth, uint16_t* normals, float* points,
                           uint32_t* inst_stats, uint32_t n_labels, oracle_stats* st);

/* Same plus the label coverage of the occlusion ratio: label_covered
 * [n_labels] = pixels each label covers with a fragment in the depth range
 * that passes its alpha test (no depth test); a 32x16 tile with more than 32
 * such labels flags them with bit 31 and adds no counts. */
int oracle_render_frame_cov(const oracle_scene* s, const float* view, const float* proj,
                            uint8_t* rgb, int32_t* inst, float* depth, uint16_t* normals, float* points,
                            uint32_t* inst_stats, uint32_t* label_covered, uint32_t n_labels,
                            oracle_stats* st);

/* Project world keypoints; visibility against a rendered depth buffer.
 * uv: [n][2], vis: [n] (0 out/behind, 1 occluded, 2 visible). */
int oracle_keypoints(const oracle_scene* s, const float* view, const float* proj,
                     const float* pts, uint32_t n, const float* depth,
                     float* uv, int32_t* vis);

/* fp32 4x4 product with the fixed summation order of the spec. */
void oracle_mat4_mul(const float* a, const float* b, float* c);

/* Render n_frames frames with `threads` OpenMP threads (cpu baseline).
 * models: optional per-frame instance transforms [n_frames][n_inst][16]. */
int oracle_render_frames(const oracle_scene* s, const float* views, const float* projs,
                         uint32_t n_frames, const float* models, uint8_t* rgb, int32_t* inst,
                         float* depth, int threads);

#ifdef __cplusplus
}
#endif
#endif
