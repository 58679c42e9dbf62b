#!/bin/bash
# A/B: k_raster tile order, squares of WxH tiles per XCD (2x2 = HEAD; 4x1 makes
# each 96-B RGB row segment quartet whole 128-B lines written from one L2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PARITY=sq41 LIBS="base sq22 sq41 sq42" REPS=3 bash tools/ab_round.sh 2>&1 | tee gpurun_out/ab_sq.txt
