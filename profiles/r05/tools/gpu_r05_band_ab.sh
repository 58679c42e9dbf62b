#!/bin/bash
# Round 5: banded binning (kBinBand; k_count / k_bin templated on banding) vs the
# build before it (libcsg_preband.so: tools/build_variant.sh preband <rev before
# the bands>) at C3 and C5, after the largest-frame and parity tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05/ab
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_max_frame.py tests/test_gpu_parity.py > gpurun_out/r05/ab/pytest_band.log 2>&1 || { tail -30 gpurun_out/r05/ab/pytest_band.log; exit 1; }
tail -1 gpurun_out/r05/ab/pytest_band.log
REPS=2 STEPS=6 FPS=2880 SKIP_LDS=1 CTR_VARIANTS="" VARIANTS="preband base" bash tools/gpu_variant_ab.sh || exit 1
mv gpurun_out/r05/ab/tile_ab.txt gpurun_out/r05/ab/band_C3.txt
REPS=3 STEPS=6 FPS=480 EXTRA="--workload C5" SKIP_LDS=1 CTR_VARIANTS="" VARIANTS="preband base" bash tools/gpu_variant_ab.sh || exit 1
mv gpurun_out/r05/ab/tile_ab.txt gpurun_out/r05/ab/band_C5.txt
