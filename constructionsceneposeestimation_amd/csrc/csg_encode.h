// csg_encode.h — host launchers of the GPU file encoders (csg_encode.hip),
// called by csg_api.cpp for csg_outputs.file_kinds.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "csg_deflate.h"

namespace csg {

// Per frame of one PNG kind: histogram, codes, header bits and sizes.
struct EncPng {
  uint32_t hist[dfl::kLitCodes + 2];
  uint32_t code[dfl::kLitCodes + 2];          // reversed code | length << 16
  uint32_t hdr[dfl::kMaxHeaderWords];         // zlib header + dynamic-block header, LSB-first bits
  uint32_t hdr_bits, adler, eob_pos, zbytes;  // zbytes: the zlib stream incl. the Adler-32
};

// Work units per frame (segments of rows): scratch arrays are [F][units].
uint32_t png_units_per_frame(uint32_t W, uint32_t H);
uint32_t csv_units_per_frame(uint32_t W, uint32_t H);
// Passes up to the sizes: fsize[f * nk + kslot] = PNG file bytes of frame f.
// rowsum, rowbits: [F][png units] scratch (rowbits become the units' bit offsets).
void launch_png_sizes(const uint8_t* img, uint32_t W, uint32_t H, uint32_t F, EncPng* png, uint2* rowsum,
                      uint32_t* rowbits, uint64_t* fsize, uint32_t nk, uint32_t kslot, hipStream_t st);
// rowlen [F][csv units] scratch (becomes the units' byte offsets); fsize as above.
void launch_csv_sizes(const float* depth, uint32_t W, uint32_t H, uint32_t F, uint32_t* rowlen, uint64_t* fsize,
                      uint32_t nk, uint32_t kslot, hipStream_t st);
// foff[n_files + 1]; zoff[2F + 1] staging offsets of the PNG frames of kind a then kind b (either may be NULL).
void launch_file_layout(const uint64_t* fsize, uint32_t n_files, uint64_t* foff, const EncPng* png_a,
                        const EncPng* png_b, uint32_t F, uint64_t* zoff, hipStream_t st);
// zbuf zeroed over the staging range first; zbase = zoff of this kind.
void launch_png_emit(const uint8_t* img, uint32_t W, uint32_t H, uint32_t F, const EncPng* png, const uint32_t* rowoff,
                     uint8_t* zbuf, const uint64_t* zbase, uint8_t* out, const uint64_t* foff, uint32_t nk,
                     uint32_t kslot, hipStream_t st);
void launch_csv_emit(const float* depth, uint32_t W, uint32_t H, uint32_t F, const uint32_t* rowoff, uint8_t* out,
                     const uint64_t* foff, uint32_t nk, uint32_t kslot, hipStream_t st);
// Point-cloud TXT: units as the CSV's (64 pixels of a row); points [F][H][W][3] f32, rgb [F][H][W][3].
void launch_pcd_sizes(const float* points, const uint8_t* rgb, uint32_t W, uint32_t H, uint32_t F, uint32_t* rowlen,
                      uint64_t* fsize, uint32_t nk, uint32_t kslot, hipStream_t st);
void launch_pcd_emit(const float* points, const uint8_t* rgb, uint32_t W, uint32_t H, uint32_t F, const uint32_t* rowoff,
                     uint8_t* out, const uint64_t* foff, uint32_t nk, uint32_t kslot, hipStream_t st);

// Quality-log depth statistics of F frames: out [F][6] (csg_outputs.depth_stats);
// scratch of depth_stats_scratch_bytes(F).
size_t depth_stats_scratch_bytes(uint32_t F);
void launch_depth_stats(const float* depth, uint32_t npx, uint32_t F, void* scratch, double* out, hipStream_t st);

}  // namespace csg
