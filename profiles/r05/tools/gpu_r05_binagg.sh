#!/bin/bash
# Round 5: wave-aggregated LDS atomics in k_count / k_bin (CSG_BIN_AGG, lane_run):
# parity through the production build, then an A/B against the per-lane build
# (libcsg_noagg.so: tools/build_variant.sh noagg - -DCSG_BIN_AGG=0) at C3 and C5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05/ab
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_sizing.py > gpurun_out/r05/pytest_binagg.log 2>&1 || { tail -30 gpurun_out/r05/pytest_binagg.log; exit 1; }
tail -1 gpurun_out/r05/pytest_binagg.log
REPS=${REPS:-3} STEPS=6 FPS=2880 SKIP_LDS=1 CTR_VARIANTS="" VARIANTS="noagg base" bash tools/gpu_variant_ab.sh || exit 1
cp gpurun_out/r05/ab/tile_ab.txt gpurun_out/r05/ab/binagg_C3.txt
rm gpurun_out/r05/ab/tile_ab.txt
REPS=2 STEPS=6 FPS=480 EXTRA="--workload C5" SKIP_LDS=1 CTR_VARIANTS="" VARIANTS="noagg base" bash tools/gpu_variant_ab.sh || exit 1
cp gpurun_out/r05/ab/tile_ab.txt gpurun_out/r05/ab/binagg_C5.txt
