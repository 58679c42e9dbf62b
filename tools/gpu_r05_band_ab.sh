#!/bin/bash
# Round 5: banded binning (kBinBand) vs the build before it (libcsg_preband.so:
# tools/build_variant.sh preband <rev before the bands>) at C3 and C5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05/ab
REPS=2 STEPS=6 FPS=2880 SKIP_LDS=1 CTR_VARIANTS="" VARIANTS="preband base" bash tools/gpu_r05_tile_ab.sh || exit 1
mv gpurun_out/r05/ab/tile_ab.txt gpurun_out/r05/ab/band_C3.txt
REPS=2 STEPS=6 FPS=480 EXTRA="--workload C5" SKIP_LDS=1 CTR_VARIANTS="" VARIANTS="preband base" bash tools/gpu_r05_tile_ab.sh || exit 1
mv gpurun_out/r05/ab/tile_ab.txt gpurun_out/r05/ab/band_C5.txt
