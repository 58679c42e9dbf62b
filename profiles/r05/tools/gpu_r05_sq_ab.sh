#!/bin/bash
# Round 5: the XCD square shape of k_raster's tile order with 32x16 tiles
# (2x2 tiles = 64x32 px, the production order; 2x4 = 64x64 px, the round-4
# footprint; 1x4, 1x2, 4x4), at the bench's launch size.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPS=${REPS:-2} STEPS=6 FPS=2880 SKIP_LDS=1 CTR_VARIANTS="" VARIANTS="${VARIANTS:-base sq24 sq14 sq12 sq44}" \
  bash tools/gpu_variant_ab.sh
