#!/bin/bash
# round-2 A/B of the k_raster level-1 / coarse-z variants (tools/build_variant.sh builds)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIBS="${LIBS:-base b0 c0 e1 f2 g1}" REPS=${REPS:-2} timeout -k 10 900 bash tools/ab_lib.sh
