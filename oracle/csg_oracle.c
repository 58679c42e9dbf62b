/*
 * CPU ORACLE — TEST INFRASTRUCTURE ONLY (see csg_oracle.h).
 *
 * Straight-line restatement of the raster spec in DESIGN.md: one frame at a
 * time, one triangle at a time, a full-frame 64-bit (depth,id) buffer.  No
 * tiling, no binning, no parallelism inside a frame — deliberately the
 * simplest program with the spec's arithmetic, so that the tiled GPU path
 * can be checked against it.
 *
 * Built with -ffp-contract=off: every float expression below is evaluated
 * exactly in the written order with IEEE-754 binary32 rounding.
 *
 * Reference anchors (generate_construction_data.py):
 *   intrinsics fx = W*f/hA, fy = H*f/vA, cx = W/2, cy = H/2 ........ :646-649
 *   clip range (0.5, 250) ............................................ :1437
 *   depth = distance_to_image_plane, inf where no hit ............... :1460, :318-321 (logger)
 *   instance mask int32, -1 background ............................... :1909-1910
 */
#include "csg_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define SUBPIX 8
#define GUARD_PX 1048576.0f
#define EMPTY_KEY 0xFFFFFFFFFFFFFFFFull

static inline float dot4(const float* r, float x, float y, float z) {
  return ((r[0] * x + r[1] * y) + r[2] * z) + r[3];
}

void oracle_mat4_mul(const float* a, const float* b, float* c) {
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j)
      c[i * 4 + j] = ((a[i * 4 + 0] * b[0 * 4 + j] + a[i * 4 + 1] * b[1 * 4 + j]) +
                      a[i * 4 + 2] * b[2 * 4 + j]) + a[i * 4 + 3] * b[3 * 4 + j];
}

static inline uint32_t fbits(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}

typedef struct { float x, y, w; } cv3;

/* Homogeneous edge coefficients of the ORIGINAL triangle: row k = v_a x v_b. */
typedef struct {
  float A[3], B[3], C[3];
  float invdet;
  int ok;
  float D[3], U[3], V[3];   /* 1/W, u/W, v/W screen planes (hom_planes) */
} hom_t;

static void hom_setup(const cv3* v, hom_t* h) {
  static const int ea[3] = {1, 2, 0}, eb[3] = {2, 0, 1};
  for (int k = 0; k < 3; ++k) {
    const cv3 a = v[ea[k]], b = v[eb[k]];
    h->A[k] = a.y * b.w - a.w * b.y;
    h->B[k] = a.w * b.x - a.x * b.w;
    h->C[k] = a.x * b.y - a.y * b.x;
  }
  const float det = (v[0].x * h->A[0] + v[0].y * h->B[0]) + v[0].w * h->C[0];
  h->ok = det != 0.0f;
  h->invdet = h->ok ? 1.0f / det : 0.0f;
}

/* Spec 5-6: the screen planes of 1/W, u/W and v/W.  With e_k = A_k x + B_k y
 * + C_k, 1/W = invdet * sum e_k and u/W = invdet * sum e_k u_k are affine:
 * D = (((A0 + A1) + A2) * invdet, ...), U = (((A0 u0 + A1 u1) + A2 u2) * invdet,
 * ...), V likewise with v. */
static void hom_planes(hom_t* h, const float uv[3][2]) {
  h->D[0] = ((h->A[0] + h->A[1]) + h->A[2]) * h->invdet;
  h->D[1] = ((h->B[0] + h->B[1]) + h->B[2]) * h->invdet;
  h->D[2] = ((h->C[0] + h->C[1]) + h->C[2]) * h->invdet;
  h->U[0] = ((h->A[0] * uv[0][0] + h->A[1] * uv[1][0]) + h->A[2] * uv[2][0]) * h->invdet;
  h->U[1] = ((h->B[0] * uv[0][0] + h->B[1] * uv[1][0]) + h->B[2] * uv[2][0]) * h->invdet;
  h->U[2] = ((h->C[0] * uv[0][0] + h->C[1] * uv[1][0]) + h->C[2] * uv[2][0]) * h->invdet;
  h->V[0] = ((h->A[0] * uv[0][1] + h->A[1] * uv[1][1]) + h->A[2] * uv[2][1]) * h->invdet;
  h->V[1] = ((h->B[0] * uv[0][1] + h->B[1] * uv[1][1]) + h->B[2] * uv[2][1]) * h->invdet;
  h->V[2] = ((h->C[0] * uv[0][1] + h->C[1] * uv[1][1]) + h->C[2] * uv[2][1]) * h->invdet;
}

static inline float plane_at(const float* P, float fx, float fy) { return (P[0] * fx + P[1] * fy) + P[2]; }

/* 1/W at the pixel centre. */
static inline float hom_invw(const hom_t* h, int px, int py) {
  return plane_at(h->D, (float)px + 0.5f, (float)py + 0.5f);
}

/* Bilinear RGBA8 fetch, repeat wrap, 8-bit fixed weights. */
static void tex_sample(const oracle_scene* s, int tid, float u, float v, int out[4]) {
  const oracle_texture* t = &s->textures[tid];
  const int tw = (int)t->width, th = (int)t->height;
  float tu = u * (float)tw - 0.5f;
  float tv = (1.0f - v) * (float)th - 0.5f;
  if (!(fabsf(tu) < 8388608.0f)) tu = 0.0f;
  if (!(fabsf(tv) < 8388608.0f)) tv = 0.0f;
  const float fu = floorf(tu), fv = floorf(tv);
  const int wx = (int)((tu - fu) * 256.0f), wy = (int)((tv - fv) * 256.0f);
  int x0 = (int)fu % tw;
  if (x0 < 0) x0 += tw;
  int y0 = (int)fv % th;
  if (y0 < 0) y0 += th;
  const int x1 = (x0 + 1 == tw) ? 0 : x0 + 1;
  const int y1 = (y0 + 1 == th) ? 0 : y0 + 1;
  const uint8_t* base = s->texels + (size_t)t->offset * 4;
  const uint8_t* c00 = base + ((size_t)y0 * tw + x0) * 4;
  const uint8_t* c10 = base + ((size_t)y0 * tw + x1) * 4;
  const uint8_t* c01 = base + ((size_t)y1 * tw + x0) * 4;
  const uint8_t* c11 = base + ((size_t)y1 * tw + x1) * 4;
  for (int c = 0; c < 4; ++c) {
    const int top = c00[c] * (256 - wx) + c10[c] * wx;
    const int bot = c01[c] * (256 - wx) + c11[c] * wx;
    out[c] = (top * (256 - wy) + bot * wy + 32768) >> 16;
  }
}

/* Triangle uid = (instance << 20) | triangle: the z-buffer tie-break id. */
#define UID_SHIFT 20

typedef struct {
  const oracle_scene* s;
  float clip[16];             /* P * V * M for the current instance */
  const oracle_mesh* m;
  const oracle_material* mat;
} inst_ctx;

static void tri_clip_coords(const inst_ctx* ic, uint32_t t, cv3 v[3], float uv[3][2]) {
  const oracle_scene* s = ic->s;
  const uint32_t* tri = s->tris + (size_t)(ic->m->tbase + t) * 3;
  for (int k = 0; k < 3; ++k) {
    const float* p = s->positions + (size_t)(ic->m->vbase + tri[k]) * 3;
    v[k].x = dot4(ic->clip + 0, p[0], p[1], p[2]);
    v[k].y = dot4(ic->clip + 4, p[0], p[1], p[2]);
    v[k].w = dot4(ic->clip + 12, p[0], p[1], p[2]);
  }
  if (uv) {
    if (ic->m->has_uv) {
      const uint32_t* ut = s->uv_tris + (size_t)(ic->m->tbase + t) * 3;
      for (int k = 0; k < 3; ++k) {
        const float* q = s->uvs + (size_t)(ic->m->uvbase + ut[k]) * 2;
        uv[k][0] = q[0];
        uv[k][1] = q[1];
      }
    } else {
      memset(uv, 0, sizeof(float) * 6);
    }
  }
}

/* Texture coordinates at the pixel centre: u = U(x, y) * (1 / (1/W)). */
static inline void interp_uv(const hom_t* h, int px, int py, float invw, float* u, float* v) {
  const float fx = (float)px + 0.5f, fy = (float)py + 0.5f, r = 1.0f / invw;
  *u = plane_at(h->U, fx, fy) * r;
  *v = plane_at(h->V, fx, fy) * r;
}

/* Label coverage for occlusion: per label, the pixels a
 * fragment of it covers (centre covered, depth in range, alpha test passed;
 * no depth test), and per 32x16 tile (k_raster's tile since round 5) the
 * labels that have such a fragment. */
#define COV_TILE_W 32
#define COV_TILE_H 16
#define COV_SLOTS 32
#define COV_UNKNOWN 0x80000000u
typedef struct {
  uint8_t* bits;        /* [n_labels][H*W] bit per pixel */
  uint8_t* tile;        /* [n_tiles][n_labels] */
  uint32_t n_labels, tiles_x, tiles_y;
} cov_t;

static int alpha_passes(const oracle_scene* s, const oracle_material* mat, const hom_t* h, int px, int py,
                        float invw) {
  if (!(mat->alpha_test && mat->texture >= 0)) return 1;
  float u, v;
  int c[4];
  interp_uv(h, px, py, invw, &u, &v);
  tex_sample(s, mat->texture, u, v, c);
  return c[3] > (int)mat->alpha_threshold;
}

/* Rasterise one screen triangle (fixed point) for the original triangle `uid`. */
static void raster_tri(const oracle_scene* s, uint64_t* zbuf, const float su[3], const float sv[3],
                       const hom_t* h, uint32_t uid, const oracle_material* mat,
                       oracle_stats* st, cov_t* cv) {
  const int W = (int)s->width, H = (int)s->height;
  int32_t x[3], y[3];
  for (int k = 0; k < 3; ++k) {
    if (!(fabsf(su[k]) < GUARD_PX) || !(fabsf(sv[k]) < GUARD_PX)) return;
    x[k] = (int32_t)rintf(su[k] * 256.0f);
    y[k] = (int32_t)rintf(sv[k] * 256.0f);
  }
  int64_t area = (int64_t)(x[1] - x[0]) * (y[2] - y[0]) - (int64_t)(x[2] - x[0]) * (y[1] - y[0]);
  if (area == 0) return;
  if (area < 0) {
    int32_t t = x[1]; x[1] = x[2]; x[2] = t;
    t = y[1]; y[1] = y[2]; y[2] = t;
  }
  int32_t xmin = x[0], xmax = x[0], ymin = y[0], ymax = y[0];
  for (int k = 1; k < 3; ++k) {
    if (x[k] < xmin) xmin = x[k];
    if (x[k] > xmax) xmax = x[k];
    if (y[k] < ymin) ymin = y[k];
    if (y[k] > ymax) ymax = y[k];
  }
  int px0 = (xmin - 128 + 255) >> 8, px1 = (xmax - 128) >> 8;
  int py0 = (ymin - 128 + 255) >> 8, py1 = (ymax - 128) >> 8;
  if (px0 < 0) px0 = 0;
  if (py0 < 0) py0 = 0;
  if (px1 > W - 1) px1 = W - 1;
  if (py1 > H - 1) py1 = H - 1;
  if (px0 > px1 || py0 > py1) return;
  st->n_raster_tris++;
  st->n_bbox_pixels += (uint64_t)(px1 - px0 + 1) * (uint64_t)(py1 - py0 + 1);
  static const int ea[3] = {1, 2, 0}, eb[3] = {2, 0, 1};
  int32_t dx[3], dy[3];
  int bias[3];
  for (int k = 0; k < 3; ++k) {
    dx[k] = x[eb[k]] - x[ea[k]];
    dy[k] = y[eb[k]] - y[ea[k]];
    bias[k] = (dy[k] < 0 || (dy[k] == 0 && dx[k] > 0)) ? 0 : -1;
  }
  const float inv_near = 1.0f / s->near_clip, inv_far = 1.0f / s->far_clip;
  for (int py = py0; py <= py1; ++py) {
    const int32_t cy = py * 256 + 128;
    for (int px = px0; px <= px1; ++px) {
      const int32_t cx = px * 256 + 128;
      int inside = 1;
      for (int k = 0; k < 3; ++k) {
        const int64_t e = (int64_t)dx[k] * (cy - y[ea[k]]) - (int64_t)dy[k] * (cx - x[ea[k]]);
        if (e + bias[k] < 0) { inside = 0; break; }
      }
      if (!inside) continue;
      st->n_covered++;
      const float invw = hom_invw(h, px, py);
      if (!(invw >= inv_far && invw <= inv_near)) continue;
      st->n_fragments++;
      if (cv) {
        const int32_t lab = s->inst_label[uid >> UID_SHIFT];
        if (lab >= 0 && (uint32_t)lab < cv->n_labels && alpha_passes(s, mat, h, px, py, invw)) {
          const size_t bit = (size_t)lab * W * H + (size_t)py * W + px;
          cv->bits[bit >> 3] |= (uint8_t)(1u << (bit & 7));
          cv->tile[((size_t)(py / COV_TILE_H) * cv->tiles_x + px / COV_TILE_W) * cv->n_labels + lab] = 1;
        }
      }
      const uint64_t key = ((uint64_t)(0xFFFFFFFFu - fbits(invw)) << 32) | uid;
      uint64_t* z = &zbuf[(size_t)py * W + px];
      if (key >= *z) { st->n_early_z_killed++; continue; }
      if (mat->alpha_test && mat->texture >= 0) {
        st->n_alpha_tests++;
        float u, v;
        int c[4];
        interp_uv(h, px, py, invw, &u, &v);
        tex_sample(s, mat->texture, u, v, c);
        if (!(c[3] > (int)mat->alpha_threshold)) { st->n_alpha_killed++; continue; }
      }
      *z = key;
    }
  }
}

static void build_clip(const oracle_scene* s, const float* view, const float* proj, uint32_t i, inst_ctx* ic) {
  float vm[16];
  oracle_mat4_mul(view, s->inst_model + (size_t)i * 16, vm);
  oracle_mat4_mul(proj, vm, ic->clip);
  ic->s = s;
  ic->m = &s->meshes[s->inst_mesh[i]];
  ic->mat = &s->materials[ic->m->material];
}

/* float -> IEEE half, round to nearest even (bit pattern). */
static uint16_t f32_to_f16(float f) {
  uint32_t x;
  memcpy(&x, &f, 4);
  const uint32_t sign = (x >> 16) & 0x8000u;
  const uint32_t e8 = (x >> 23) & 0xffu;
  uint32_t mant = x & 0x7fffffu;
  if (e8 == 0xffu) return (uint16_t)(sign | 0x7c00u | (mant ? 0x200u : 0u));
  const int32_t e = (int32_t)e8 - 127 + 15;
  if (e >= 31) return (uint16_t)(sign | 0x7c00u);
  if (e <= 0) {                      /* half subnormal or zero */
    if (e < -10) return (uint16_t)sign;
    mant |= 0x800000u;
    const uint32_t shift = (uint32_t)(14 - e);
    uint32_t hm = mant >> shift;
    const uint32_t rem = mant & ((1u << shift) - 1u), halfway = 1u << (shift - 1u);
    if (rem > halfway || (rem == halfway && (hm & 1u))) hm++;
    return (uint16_t)(sign | hm);
  }
  uint32_t h = sign | ((uint32_t)e << 10) | (mant >> 13);
  const uint32_t rem = mant & 0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;
  return (uint16_t)h;
}

/* Per-frame unprojection constants: camera-to-world rotation (transpose of
 * the view rotation), camera position -R^T t, fx, fy, cx, cy read back from
 * the pixel projection. */
static void frame_camera(const float* V, const float* P, float* cam) {
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) cam[i * 3 + j] = V[j * 4 + i];
    cam[9 + i] = -((V[0 * 4 + i] * V[3] + V[1 * 4 + i] * V[7]) + V[2 * 4 + i] * V[11]);
  }
  cam[12] = P[0];
  cam[13] = -P[5];
  cam[14] = -P[2];
  cam[15] = -P[6];
}

/* World point on the ray through the pixel centre at distance-to-image-plane d
 * (the depth_to_pointcloud step, generate_construction_data.py:616-711, in
 * the USD camera convention). */
static void unproject(const float* cam, int px, int py, float d, float* out) {
  const float a = ((float)px + 0.5f) - cam[14], b = ((float)py + 0.5f) - cam[15];
  const float xc = (a * d) / cam[12], yc = -((b * d) / cam[13]), zc = -d;
  for (int i = 0; i < 3; ++i) out[i] = ((cam[i * 3 + 0] * xc + cam[i * 3 + 1] * yc) + cam[i * 3 + 2] * zc) + cam[9 + i];
}

int oracle_render_frame(const oracle_scene* s, const float* view, const float* proj,
                        uint8_t* rgb, int32_t* inst, float* depth,
                        uint32_t* inst_stats, uint32_t n_labels, oracle_stats* st_out) {
  return oracle_render_frame_ex(s, view, proj, rgb, inst, depth, NULL, NULL, inst_stats, n_labels, st_out);
}

int oracle_render_frame_ex(const oracle_scene* s, const float* view, const float* proj,
                           uint8_t* rgb, int32_t* inst, float* depth, uint16_t* normals, float* points,
                           uint32_t* inst_stats, uint32_t n_labels, oracle_stats* st_out) {
  return oracle_render_frame_cov(s, view, proj, rgb, inst, depth, normals, points, inst_stats, NULL, n_labels,
                                 st_out);
}

/* covered[l] from the coverage bits: tiles holding more than COV_SLOTS labels
 * flag their labels unknown and add no counts (the GPU's tile table). */
static void cov_finish(const cov_t* cv, int W, int H, uint32_t* covered) {
  for (uint32_t l = 0; l < cv->n_labels; ++l) covered[l] = 0;
  for (uint32_t ty = 0; ty < cv->tiles_y; ++ty) {
    for (uint32_t tx = 0; tx < cv->tiles_x; ++tx) {
      const uint8_t* tl = cv->tile + ((size_t)ty * cv->tiles_x + tx) * cv->n_labels;
      uint32_t n = 0;
      for (uint32_t l = 0; l < cv->n_labels; ++l) n += tl[l];
      for (uint32_t l = 0; l < cv->n_labels; ++l) {
        if (!tl[l]) continue;
        if (n > COV_SLOTS) { covered[l] |= COV_UNKNOWN; continue; }
        uint32_t cnt = 0;
        for (int py = (int)ty * COV_TILE_H; py < (int)(ty + 1) * COV_TILE_H && py < H; ++py)
          for (int px = (int)tx * COV_TILE_W; px < (int)(tx + 1) * COV_TILE_W && px < W; ++px) {
            const size_t bit = (size_t)l * W * H + (size_t)py * W + px;
            cnt += (cv->bits[bit >> 3] >> (bit & 7)) & 1u;
          }
        covered[l] += cnt;
      }
    }
  }
}

int oracle_render_frame_cov(const oracle_scene* s, const float* view, const float* proj,
                            uint8_t* rgb, int32_t* inst, float* depth, uint16_t* normals, float* points,
                            uint32_t* inst_stats, uint32_t* label_covered, uint32_t n_labels,
                            oracle_stats* st_out) {
  const int W = (int)s->width, H = (int)s->height;
  uint64_t* zbuf = (uint64_t*)malloc((size_t)W * H * sizeof(uint64_t));
  if (!zbuf) return -1;
  cov_t cov_store, *cv = NULL;
  if (label_covered && n_labels) {
    cov_store.n_labels = n_labels;
    cov_store.tiles_x = (uint32_t)(W + COV_TILE_W - 1) / COV_TILE_W;
    cov_store.tiles_y = (uint32_t)(H + COV_TILE_H - 1) / COV_TILE_H;
    cov_store.bits = (uint8_t*)calloc(((size_t)n_labels * W * H + 7) / 8, 1);
    cov_store.tile = (uint8_t*)calloc((size_t)cov_store.tiles_x * cov_store.tiles_y * n_labels, 1);
    if (!cov_store.bits || !cov_store.tile) {
      free(cov_store.bits); free(cov_store.tile); free(zbuf);
      return -1;
    }
    cv = &cov_store;
  }
  for (size_t i = 0; i < (size_t)W * H; ++i) zbuf[i] = EMPTY_KEY;
  oracle_stats st;
  memset(&st, 0, sizeof(st));
  int limit = s->n_inst >= (1u << (32 - UID_SHIFT));
  for (uint32_t i = 0; i < s->n_inst; ++i) limit |= s->meshes[s->inst_mesh[i]].ntris >= (1u << UID_SHIFT);
  if (limit) {
    if (cv) { free(cv->bits); free(cv->tile); }
    free(zbuf);
    return -2;
  }
  const float near = s->near_clip, far = s->far_clip;
  const float Wf = (float)W, Hf = (float)H;

  for (uint32_t i = 0; i < s->n_inst; ++i) {
    inst_ctx ic;
    build_clip(s, view, proj, i, &ic);
    for (uint32_t t = 0; t < ic.m->ntris; ++t) {
      st.n_tris_in++;
      cv3 v[3];
      float uv[3][2];
      tri_clip_coords(&ic, t, v, uv);
      /* trivial rejects against the homogeneous frustum */
      int out_near = 1, out_far = 1, out_l = 1, out_r = 1, out_t = 1, out_b = 1;
      for (int k = 0; k < 3; ++k) {
        out_near &= v[k].w < near;
        out_far &= v[k].w > far;
        out_l &= v[k].x < 0.0f;
        out_r &= v[k].x > Wf * v[k].w;
        out_t &= v[k].y < 0.0f;
        out_b &= v[k].y > Hf * v[k].w;
      }
      if (out_near | out_far | out_l | out_r | out_t | out_b) { st.n_culled++; continue; }
      hom_t h;
      hom_setup(v, &h);
      if (!h.ok) { st.n_culled++; continue; }
      hom_planes(&h, uv);
      const uint32_t uid = (i << UID_SHIFT) | t;
      const int all_in = v[0].w >= near && v[1].w >= near && v[2].w >= near;
      if (all_in) {
        float su[3], sv[3];
        for (int k = 0; k < 3; ++k) {   /* spec 3: one reciprocal per vertex, u = X * (1/W) */
          const float rw = 1.0f / v[k].w;
          su[k] = v[k].x * rw;
          sv[k] = v[k].y * rw;
        }
        raster_tri(s, zbuf, su, sv, &h, uid, ic.mat, &st, cv);
      } else {
        /* Sutherland-Hodgman against W >= near, edges v0->v1, v1->v2, v2->v0 */
        st.n_clipped++;
        cv3 q[4];
        int nq = 0;
        for (int k = 0; k < 3; ++k) {
          const cv3 a = v[k], b = v[(k + 1) % 3];
          const int ain = a.w >= near, bin = b.w >= near;
          if (ain) q[nq++] = a;
          if (ain != bin) {
            const float tt = (near - a.w) / (b.w - a.w);
            cv3 r;
            r.x = a.x + tt * (b.x - a.x);
            r.y = a.y + tt * (b.y - a.y);
            r.w = near;
            q[nq++] = r;
          }
        }
        for (int f = 1; f + 1 < nq; ++f) {
          const cv3 tri3[3] = {q[0], q[f], q[f + 1]};
          float su[3], sv[3];
          for (int k = 0; k < 3; ++k) {
            const float rw = 1.0f / tri3[k].w;
            su[k] = tri3[k].x * rw;
            sv[k] = tri3[k].y * rw;
          }
          raster_tri(s, zbuf, su, sv, &h, uid, ic.mat, &st, cv);
        }
      }
    }
  }

  if (cv) {
    cov_finish(cv, W, H, label_covered);
    free(cv->bits);
    free(cv->tile);
  }
  /* resolve */
  float cam[16];
  frame_camera(view, proj, cam);
  if (inst_stats && n_labels) {
    for (uint32_t l = 0; l < n_labels; ++l) {
      inst_stats[l * 5 + 0] = 0;
      inst_stats[l * 5 + 1] = 0xFFFFFFFFu;
      inst_stats[l * 5 + 2] = 0xFFFFFFFFu;
      inst_stats[l * 5 + 3] = 0;
      inst_stats[l * 5 + 4] = 0;
    }
  }
  for (int py = 0; py < H; ++py) {
    for (int px = 0; px < W; ++px) {
      const size_t p = (size_t)py * W + px;
      const uint64_t key = zbuf[p];
      if (key == EMPTY_KEY) {
        if (rgb) { rgb[p * 3 + 0] = s->sky[0]; rgb[p * 3 + 1] = s->sky[1]; rgb[p * 3 + 2] = s->sky[2]; }
        if (inst) inst[p] = -1;
        if (depth) depth[p] = INFINITY;
        if (normals) normals[p * 3 + 0] = normals[p * 3 + 1] = normals[p * 3 + 2] = 0;
        if (points) points[p * 3 + 0] = points[p * 3 + 1] = points[p * 3 + 2] = NAN;
        continue;
      }
      const uint32_t uid = (uint32_t)key;
      const int i = (int)(uid >> UID_SHIFT);
      const uint32_t t = uid & ((1u << UID_SHIFT) - 1u);
      inst_ctx ic;
      build_clip(s, view, proj, (uint32_t)i, &ic);
      cv3 v[3];
      float uv[3][2];
      tri_clip_coords(&ic, t, v, uv);
      hom_t h;
      hom_setup(v, &h);
      hom_planes(&h, uv);
      const float invw = hom_invw(&h, px, py);
      const int32_t label = s->inst_label[i];
      if (depth) depth[p] = 1.0f / invw;
      if (points) unproject(cam, px, py, 1.0f / invw, points + p * 3);
      if (inst) inst[p] = label;
      if (inst_stats && label >= 0 && (uint32_t)label < n_labels) {
        uint32_t* q = inst_stats + (size_t)label * 5;
        q[0]++;
        if ((uint32_t)px < q[1]) q[1] = (uint32_t)px;
        if ((uint32_t)py < q[2]) q[2] = (uint32_t)py;
        if ((uint32_t)px > q[3]) q[3] = (uint32_t)px;
        if ((uint32_t)py > q[4]) q[4] = (uint32_t)py;
      }
      if (!rgb && !normals) continue;
      int alb[3];
      const oracle_material* mat = ic.mat;
      if (mat->texture >= 0 && ic.m->has_uv) {
        float u, vv;
        int c[4];
        interp_uv(&h, px, py, invw, &u, &vv);
        tex_sample(s, mat->texture, u, vv, c);
        for (int k = 0; k < 3; ++k) alb[k] = (c[k] * mat->base[k] + 127) / 255;
      } else {
        for (int k = 0; k < 3; ++k) alb[k] = mat->base[k];
      }
      /* flat two-sided Lambert from the world-space face normal */
      const float* M = s->inst_model + (size_t)i * 16;
      const uint32_t* tri = s->tris + (size_t)(ic.m->tbase + t) * 3;
      float pw[3][3];
      for (int k = 0; k < 3; ++k) {
        const float* q = s->positions + (size_t)(ic.m->vbase + tri[k]) * 3;
        pw[k][0] = dot4(M + 0, q[0], q[1], q[2]);
        pw[k][1] = dot4(M + 4, q[0], q[1], q[2]);
        pw[k][2] = dot4(M + 8, q[0], q[1], q[2]);
      }
      const float e1x = pw[1][0] - pw[0][0], e1y = pw[1][1] - pw[0][1], e1z = pw[1][2] - pw[0][2];
      const float e2x = pw[2][0] - pw[0][0], e2y = pw[2][1] - pw[0][1], e2z = pw[2][2] - pw[0][2];
      const float nx = e1y * e2z - e1z * e2y;
      const float ny = e1z * e2x - e1x * e2z;
      const float nz = e1x * e2y - e1y * e2x;
      const float nn = (nx * nx + ny * ny) + nz * nz;
      float c = 0.0f;
      uint16_t nh[3] = {0, 0, 0};
      if (nn > 0.0f) {
        const float len = sqrtf(nn);
        const float d = (nx * s->sun_dir[0] + ny * s->sun_dir[1]) + nz * s->sun_dir[2];
        c = fabsf(d / len);
        /* two-sided normal: det(clip) < 0 exactly when the face points at the camera */
        const float sg = h.invdet < 0.0f ? 1.0f : -1.0f;
        /* + 0.0f: no negative zeros in the output */
        nh[0] = f32_to_f16(sg * (nx / len) + 0.0f);
        nh[1] = f32_to_f16(sg * (ny / len) + 0.0f);
        nh[2] = f32_to_f16(sg * (nz / len) + 0.0f);
      }
      if (normals) { normals[p * 3 + 0] = nh[0]; normals[p * 3 + 1] = nh[1]; normals[p * 3 + 2] = nh[2]; }
      if (!rgb) continue;
      for (int k = 0; k < 3; ++k) {
        const float shade = s->ambient[k] + s->sun[k] * c;
        int q = (int)(shade * 256.0f + 0.5f);
        if (q < 0) q = 0;
        if (q > 65535) q = 65535;
        int o = (alb[k] * q + 128) >> 8;
        rgb[p * 3 + k] = (uint8_t)(o > 255 ? 255 : o);
      }
    }
  }
  free(zbuf);
  if (st_out) *st_out = st;
  return 0;
}

int oracle_keypoints(const oracle_scene* s, const float* view, const float* proj,
                     const float* pts, uint32_t n, const float* depth, float* uv, int32_t* vis) {
  float pv[16];
  oracle_mat4_mul(proj, view, pv);
  const float Wf = (float)s->width, Hf = (float)s->height;
  for (uint32_t k = 0; k < n; ++k) {
    const float* p = pts + (size_t)k * 3;
    const float X = dot4(pv + 0, p[0], p[1], p[2]);
    const float Y = dot4(pv + 4, p[0], p[1], p[2]);
    const float Wc = dot4(pv + 12, p[0], p[1], p[2]);
    if (!(Wc >= s->near_clip)) {
      uv[k * 2 + 0] = -1.0f;
      uv[k * 2 + 1] = -1.0f;
      vis[k] = 0;
      continue;
    }
    const float u = X / Wc, v = Y / Wc;
    uv[k * 2 + 0] = u;
    uv[k * 2 + 1] = v;
    if (!(u >= 0.0f && u < Wf && v >= 0.0f && v < Hf)) { vis[k] = 0; continue; }
    const int px = (int)u, py = (int)v;
    const float d = depth ? depth[(size_t)py * s->width + px] : INFINITY;
    vis[k] = (Wc <= d) ? 2 : 1;
  }
  return 0;
}

int oracle_render_frames(const oracle_scene* s, const float* views, const float* projs,
                         uint32_t n_frames, const float* models, uint8_t* rgb, int32_t* inst, float* depth,
                         int threads) {
  const size_t npx = (size_t)s->width * s->height;
  int rc = 0;
#pragma omp parallel for num_threads(threads) schedule(dynamic, 1) reduction(| : rc)
  for (int f = 0; f < (int)n_frames; ++f) {
    oracle_scene sf = *s;
    if (models) sf.inst_model = models + (size_t)f * s->n_inst * 16;
    rc |= oracle_render_frame(&sf, views + (size_t)f * 16, projs + (size_t)f * 16,
                              rgb ? rgb + npx * 3 * f : NULL, inst ? inst + npx * f : NULL,
                              depth ? depth + npx * f : NULL, NULL, 0, NULL);
  }
  return rc;
}
