#!/bin/bash
# CPU side of tools/gpu_variant_ab.sh: the tile-shape variants of libcsg.so
# (working-tree kernels; LDS per workgroup sized for 7 waves per SIMD) and
# their ablation / profiling-counter builds.
set -e
cd "$(dirname "$0")/.."
B=tools/build_variant.sh
S108="-DCSG_STAGE=108 -DCSG_COV_STAGE=56 -DCSG_SHADE_SLOTS=104"
W64="-DCSG_TILE_W=64 -DCSG_TILE_H=16 $S108"
W32="-DCSG_TILE_W=32 -DCSG_TILE_H=16 -DCSG_STAGE=60 -DCSG_COV_STAGE=32 -DCSG_SHADE_SLOTS=64 -DCSG_LDS_LABELS=64"
W16="-DCSG_TILE_W=16 -DCSG_TILE_H=16 -DCSG_STAGE=28 -DCSG_COV_STAGE=12 -DCSG_SHADE_SLOTS=28 -DCSG_LDS_LABELS=64"
$B s108 - $S108 &
$B w64h16 - $W64 &
$B w32h16 - $W32 &
$B w16h16 - $W16 &
wait
$B abl - -DCSG_ABLATION=1 &
$B abl_w64h16 - -DCSG_ABLATION=1 $W64 &
$B abl_w32h16 - -DCSG_ABLATION=1 $W32 &
$B abl_w16h16 - -DCSG_ABLATION=1 $W16 &
wait
