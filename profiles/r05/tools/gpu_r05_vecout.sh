#!/bin/bash
# Round 5: vector stores of the per-pixel outputs (CSG_VEC_OUT) -- the GPU suite
# through the production build, then an A/B against libcsg_novec.so
# (tools/build_variant.sh novec - -DCSG_VEC_OUT=0) at C5 and C3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out/r05/ab
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r05/ab/pytest_vecout.log 2>&1 || { tail -40 gpurun_out/r05/ab/pytest_vecout.log; exit 1; }
tail -1 gpurun_out/r05/ab/pytest_vecout.log
REPS=3 STEPS=6 FPS=480 EXTRA="--workload C5" SKIP_LDS=1 CTR_VARIANTS="" VARIANTS="novec base" bash tools/gpu_variant_ab.sh || exit 1
mv gpurun_out/r05/ab/tile_ab.txt gpurun_out/r05/ab/vecout_C5.txt
REPS=2 STEPS=6 FPS=2880 SKIP_LDS=1 CTR_VARIANTS="" VARIANTS="novec base" bash tools/gpu_variant_ab.sh || exit 1
mv gpurun_out/r05/ab/tile_ab.txt gpurun_out/r05/ab/vecout_C3.txt
