/*
 * csg_io.h — C ABI of libcsgio.so, the host-side writers of the frame
 * generator's on-disk formats.  Plain C99, host only (no GPU).  Every entry
 * point returns 0 on success, a negative errno-style code on failure, and is
 * thread-safe (no shared state), so a pool of host threads can encode frames
 * in parallel while the GPU renders the next batch.
 *
 * What each writer replaces in the reference
 * (xander683/ConstructionScenePoseEstimation, generate_construction_data.py):
 *
 *   csgio_write_png_rgb ........ cv2.imwrite of the RGB frame           :1672-1673
 *   csgio_write_npy ............ np.save of the instance mask / depth   :2066-2069, :1687
 *   csgio_write_depth_csv ...... np.savetxt(depth, fmt="%.6f", " ")     :1688
 *   csgio_write_pointcloud_txt . np.savetxt(xyzrgb, fmt="%.6f", " ",
 *                                header="x y z r g b", comments="")     :769-770
 *   csgio_depth_stats .......... DataQualityLogger.log_depth's counts   :318-341
 *   csgio_write_label_json ..... save_label_json(json.dump indent=2) of
 *                                the frame's label record            :608-613, :2056-2064
 *
 * The text writers produce byte-identical output to the numpy calls (values
 * are formatted from their float64 value with "%.6f" semantics).
 */
#ifndef CSG_IO_H
#define CSG_IO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CSGIO_ABI_VERSION 4

int csgio_abi_version(void);

/* 8-bit RGB PNG (filter Sub on every row, zlib level 0..9; strategy 0 =
 * zlib default, 1 = run-length matches only (Z_RLE: about 2x faster on
 * rendered frames, ~2% larger), 2 = Huffman only). */
int csgio_write_png_rgb(const char* path, const uint8_t* rgb, uint32_t width, uint32_t height, int level,
                        int strategy);

/* NPY v1.0 file: descr e.g. "<i4", "<f4", "<f2", "|u1"; C order. */
int csgio_write_npy(const char* path, const void* data, uint64_t nbytes, const char* descr, const uint64_t* shape,
                    uint32_t ndim);

/* H rows of W space-separated "%.6f" values (np.savetxt of a float32 image). */
int csgio_write_depth_csv(const char* path, const float* depth, uint32_t width, uint32_t height);

/* One pass over a depth image (the quality log's depth entry, GDP:318-341):
 * out[0] valid pixels (finite, > 0), out[1] zero pixels, out[2] infinite
 * pixels, out[3] sum of the valid depths (float64), out[4] / out[5] min / max
 * of the valid depths (0 if none). */
int csgio_depth_stats(const float* depth, uint64_t n, double* out);

/* "x y z r g b" header, then one "%.6f" row per pixel whose point is not NaN
 * (xyz: [n][3] float32 world points, rgb: [n][3] uint8). */
int csgio_write_pointcloud_txt(const char* path, const float* xyz, const uint8_t* rgb, uint64_t n);

/* One frame's label file, byte-identical to save_label_json(label_record(...))
 * of constructionsceneposeestimation_amd/labels.py (json.dump indent=2,
 * ensure_ascii=False; floats as Python's repr), built from the frame's arrays
 * without the Python interpreter.  The fixed parts come pre-rendered as JSON
 * text: `camera_params` and `class_mapping` as values at nesting level 1,
 * `obj_head[j]` as the fields of object j (inst_idx ... prim_path) indented
 * for level 3 ("      " before the first key), `kp_name[k]` as JSON string
 * literals.  Objects with no visible pixel (inst_stats[label][0] == 0, or a
 * label past n_labels) are left out, as label_record does, unless
 * obj_listed[j] is 1 (the "frustum" object list: the object's 3D box meets the
 * view frustum): then it is written with pixel_count 0, bbox_2d [-1, -1, -1,
 * -1] and occlusion_ratio 1.0 (coverage known) or -1.0 (unknown). */
typedef struct {
  uint32_t frame_id, height, width;
  uint32_t n_objects, n_labels, n_kp;
  const double* camera_pose;          /* [7] x y z qx qy qz qw */
  const char* camera_params;          /* JSON value text, level 1 */
  const char* class_mapping;          /* JSON value text, level 1 */
  const char* const* obj_head;        /* [n_objects] */
  const int32_t* obj_label;           /* [n_objects] inst_idx: row of inst_stats / covered */
  const uint32_t* obj_kp_off;         /* [n_objects + 1] into obj_kp (keypoints of object j, table order) */
  const uint32_t* obj_kp;             /* keypoint indices */
  const uint32_t* inst_stats;         /* [n_labels][5] pixels, minx, miny, maxx, maxy */
  const uint32_t* covered;            /* [n_labels] label coverage (csg_outputs.label_covered), or NULL */
  const float* kp_uv;                 /* [n_kp][2] */
  const int32_t* kp_vis;              /* [n_kp] */
  const char* const* kp_name;         /* [n_kp] */
  const uint8_t* obj_listed;          /* [n_objects] 1: listed without visible pixels, or NULL */
} csgio_label;

int csgio_write_label_json(const char* path, const csgio_label* label);

#ifdef __cplusplus
}
#endif
#endif /* CSG_IO_H */
