#!/bin/bash
# Round 5: 32x16 tiles at the bench's default launch size (2,880 frames per
# step): the 7-wave and 6-wave builds and the k_count / k_bin block count
# (CSG_BINBLOCKS), against the 32x32 production build.  Z-buffer swizzled in all.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPS=${REPS:-2} STEPS=6 FPS=2880 SKIP_LDS=1 CTR_VARIANTS="" \
  VARIANTS="${VARIANTS:-base w32h16:CSG_BINBLOCKS=16 w32h16w6:CSG_BINBLOCKS=16 w32h16:CSG_BINBLOCKS=8 w32h16:CSG_BINBLOCKS=24}" \
  bash tools/gpu_variant_ab.sh
