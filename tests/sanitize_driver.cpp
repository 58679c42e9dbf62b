// Host code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY §5:
// sanitizers on the CPU side): the C oracle (oracle/csg_oracle.c) renders a
// synthetic scene with every output and edge case its callers meet (alpha
// card with a wrapping texture, a box, a triangle through the near plane,
// sub-pixel and far-off triangles, ragged frame size, OpenMP frames), and the
// host writers (csg_io.cpp) write every format with edge values (inf, nan,
// -0, 3.4e38; NaN / inf doubles in the label JSON).  Built and run by
// tests/test_sanitize.py; any sanitizer report aborts with a non-zero status.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../include/csg_io.h"
#include "../oracle/csg_oracle.h"

static void look(float* view, float* proj, float cx, float cy, float cz, uint32_t W, uint32_t H) {
  // camera at (cx, cy, cz) looking along -Z (USD camera), +Y up; pixel projection
  std::memset(view, 0, 16 * sizeof(float));
  view[0] = view[5] = view[10] = view[15] = 1.0f;
  view[3] = -cx;
  view[7] = -cy;
  view[11] = -cz;
  const float f = (float)W * 12.0f / 25.0f, cxp = W * 0.5f, cyp = H * 0.5f;
  std::memset(proj, 0, 16 * sizeof(float));
  proj[0] = f;   proj[2] = -cxp;   // u*w = f*x - cx*z
  proj[5] = -f;  proj[6] = -cyp;   // v*w = -f*y - cy*z
  proj[14] = -1.0f;                // w = -z
  proj[10] = -1.0f;
}

int main() {
  const uint32_t W = 203, H = 117;
  // geometry: mesh 0 = alpha card (2 tris, uvs wrapping 3x), mesh 1 = unit
  // box (12 tris), mesh 2 = loose triangles (near-plane crossing, sub-pixel,
  // far-off vertices)
  std::vector<float> pos = {
      -1, -1, 0, 1, -1, 0, 1, 1, 0, -1, 1, 0,                                           // card
      -0.5f, -0.5f, -0.5f, 0.5f, -0.5f, -0.5f, 0.5f, 0.5f, -0.5f, -0.5f, 0.5f, -0.5f,  // box
      -0.5f, -0.5f, 0.5f, 0.5f, -0.5f, 0.5f, 0.5f, 0.5f, 0.5f, -0.5f, 0.5f, 0.5f,
      0, 0, 4.8f, 0.3f, 0, 3.0f, 0, 0.3f, 3.0f,                                       // through near
      0.001f, 0.001f, 0, 0.0011f, 0.001f, 0, 0.001f, 0.0011f, 0,                        // sub-pixel
      -3000, -2000, -10, 4000, -1, -12, 1, 5000, -11};                                  // far-off
  std::vector<uint32_t> tris = {0, 1, 2, 0, 2, 3,
                                0, 2, 1, 0, 3, 2, 4, 5, 6, 4, 6, 7, 0, 1, 5, 0, 5, 4,
                                1, 2, 6, 1, 6, 5, 2, 3, 7, 2, 7, 6, 3, 0, 4, 3, 4, 7,
                                0, 1, 2, 3, 4, 5, 6, 7, 8};
  std::vector<float> uvs = {0, 0, 3, 0, 3, 3, 0, 3};
  std::vector<uint32_t> uv_tris = {0, 1, 2, 0, 2, 3};
  const oracle_mesh meshes[3] = {{0, 0, 2, 0, 1, 0}, {4, 2, 12, 0, 0, 1}, {12, 14, 3, 0, 0, 2}};
  // texture: 5x3 RGBA8 with mixed alpha (non-power-of-two)
  std::vector<uint8_t> texels(5 * 3 * 4);
  for (size_t k = 0; k < texels.size(); ++k) texels[k] = (uint8_t)(k * 37u);
  const oracle_texture tex = {0, 5, 3, 0};
  const oracle_material mats[3] = {{{200, 180, 160, 255}, 0, 1, 100}, {{90, 120, 200, 255}, -1, 0, 0},
                                   {{255, 255, 255, 255}, -1, 0, 0}};
  // instances: card twice (one behind the box), box, loose triangles
  std::vector<float> models(4 * 16, 0.0f);
  const float tx[4][3] = {{0, 0, -4}, {0.3f, 0.2f, -6}, {0.2f, -0.1f, -5}, {0, 0, 0}};
  for (int i = 0; i < 4; ++i) {
    float* M = &models[16 * i];
    M[0] = M[5] = M[10] = M[15] = 1.0f;
    M[3] = tx[i][0];
    M[7] = tx[i][1];
    M[11] = tx[i][2];
  }
  const uint32_t inst_mesh[4] = {0, 0, 1, 2};
  const int32_t inst_label[4] = {0, 1, 2, -1};
  const uint32_t inst_tri_base[5] = {0, 2, 4, 16, 19};
  oracle_scene s{};
  s.positions = pos.data();
  s.tris = tris.data();
  s.uvs = uvs.data();
  s.uv_tris = uv_tris.data();
  s.meshes = meshes;
  s.n_meshes = 3;
  s.inst_model = models.data();
  s.inst_mesh = inst_mesh;
  s.inst_label = inst_label;
  s.inst_tri_base = inst_tri_base;
  s.n_inst = 4;
  s.materials = mats;
  s.n_materials = 3;
  s.texels = texels.data();
  s.textures = &tex;
  s.n_textures = 1;
  const float amb[3] = {0.3f, 0.35f, 0.4f}, sun[3] = {0.7f, 0.7f, 0.6f}, sd[3] = {0.3f, 0.5f, 0.81f};
  for (int k = 0; k < 3; ++k) {
    s.ambient[k] = amb[k];
    s.sun[k] = sun[k];
    s.sun_dir[k] = sd[k];
  }
  s.sky[0] = 120; s.sky[1] = 160; s.sky[2] = 220; s.sky[3] = 255;
  s.width = W;
  s.height = H;
  s.near_clip = 0.5f;
  s.far_clip = 250.0f;

  const uint32_t npx = W * H, nl = 3;
  std::vector<uint8_t> rgb(npx * 3);
  std::vector<int32_t> inst(npx);
  std::vector<float> depth(npx), points(npx * 3);
  std::vector<uint16_t> normals(npx * 3);
  std::vector<uint32_t> stats(nl * 5), cov(nl);
  float view[16], proj[16];
  look(view, proj, 0.1f, 0.05f, 5.0f, W, H);
  oracle_stats st{};
  if (oracle_render_frame_cov(&s, view, proj, rgb.data(), inst.data(), depth.data(), normals.data(), points.data(),
                              stats.data(), cov.data(), nl, &st))
    return 2;
  if (st.n_fragments == 0 || st.n_alpha_tests == 0) return 3;
  const float kp[3 * 3] = {0, 0, -4, 0.2f, -0.1f, -5, 100, 100, 100};
  float uv[6];
  int32_t vis[3];
  if (oracle_keypoints(&s, view, proj, kp, 3, depth.data(), uv, vis)) return 4;
  // two frames on two OpenMP threads, per-frame models
  float views[32], projs[32];
  std::memcpy(views, view, sizeof view);
  std::memcpy(projs, proj, sizeof proj);
  look(views + 16, projs + 16, -0.3f, 0.0f, 3.0f, W, H);
  std::vector<float> fm(2 * models.size());
  std::memcpy(fm.data(), models.data(), models.size() * 4);
  std::memcpy(fm.data() + models.size(), models.data(), models.size() * 4);
  std::vector<uint8_t> rgb2(2 * npx * 3);
  std::vector<int32_t> inst2(2 * npx);
  std::vector<float> depth2(2 * npx);
  if (oracle_render_frames(&s, views, projs, 2, fm.data(), rgb2.data(), inst2.data(), depth2.data(), 2)) return 5;

  // writers, with edge values
  const std::string dir = SAN_TMPDIR;
  depth[0] = INFINITY;
  depth[1] = -INFINITY;
  depth[2] = NAN;
  depth[3] = -0.0f;
  depth[4] = 3.4e38f;
  depth[5] = 1e-30f;
  if (csgio_write_png_rgb((dir + "/a.png").c_str(), rgb.data(), W, H, 1, 1)) return 6;
  if (csgio_write_png_rgb((dir + "/b.png").c_str(), rgb.data(), W, H, 6, 0)) return 7;
  const uint64_t shape[2] = {H, W};
  if (csgio_write_npy((dir + "/m.npy").c_str(), inst.data(), npx * 4ull, "<i4", shape, 2)) return 8;
  if (csgio_write_depth_csv((dir + "/d.csv").c_str(), depth.data(), W, H)) return 9;
  points[0] = -3.4e38f;
  points[1] = 1e20f;
  if (csgio_write_pointcloud_txt((dir + "/p.txt").c_str(), points.data(), rgb.data(), npx)) return 10;
  double ds[6];
  if (csgio_depth_stats(depth.data(), npx, ds)) return 11;
  // label JSON: two objects, keypoints, coverage with the unknown flag
  const double pose[7] = {1.5, -2.25, NAN, 0.0, -0.0, INFINITY, 1e-310};
  const char* heads[2] = {"      \"inst_idx\": 0", "      \"inst_idx\": 1"};
  const int32_t obj_label[2] = {0, 1};
  const uint32_t kp_off[3] = {0, 2, 3}, kp_idx[3] = {0, 1, 2};
  const uint32_t covered[3] = {cov[0], cov[1] | 0x80000000u, cov[2]};
  const float kp_uv[6] = {1.0f, 2.5f, NAN, -INFINITY, 1e30f, -0.0f};
  const int32_t kp_vis[3] = {2, 1, 0};
  const char* kp_name[3] = {"\"c0\"", "\"c1\"", "\"centre\""};
  const uint8_t listed[2] = {1, 1};
  csgio_label L{};
  L.frame_id = 7;
  L.height = H;
  L.width = W;
  L.n_objects = 2;
  L.n_labels = nl;
  L.n_kp = 3;
  L.camera_pose = pose;
  L.camera_params = "{}";
  L.class_mapping = "{}";
  L.obj_head = heads;
  L.obj_label = obj_label;
  L.obj_kp_off = kp_off;
  L.obj_kp = kp_idx;
  L.inst_stats = stats.data();
  L.covered = covered;
  L.kp_uv = kp_uv;
  L.kp_vis = kp_vis;
  L.kp_name = kp_name;
  L.obj_listed = listed;
  if (csgio_write_label_json((dir + "/l.json").c_str(), &L)) return 12;
  L.covered = nullptr;
  L.obj_listed = nullptr;
  if (csgio_write_label_json((dir + "/l2.json").c_str(), &L)) return 13;
  std::printf("sanitize driver ok: %llu fragments, %llu alpha tests\n", (unsigned long long)st.n_fragments,
              (unsigned long long)st.n_alpha_tests);
  return 0;
}
