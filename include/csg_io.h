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

#define CSGIO_ABI_VERSION 2

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

#ifdef __cplusplus
}
#endif
#endif /* CSG_IO_H */
