#!/bin/bash
# Round 5: binning blocks per frame at 4K (C5: 16,200 tiles of 32x16), where the
# [blocks][tiles] count grid dominates k_count / k_colscan / k_bin.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPS=${REPS:-2} STEPS=4 FPS=480 SKIP_LDS=1 CTR_VARIANTS="" EXTRA="--workload C5 --verify-frames 4" \
  VARIANTS="base:CSG_BINBLOCKS=16 base:CSG_BINBLOCKS=8 base:CSG_BINBLOCKS=4 base:CSG_BINBLOCKS=2" bash tools/gpu_variant_ab.sh
