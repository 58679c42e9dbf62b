#!/bin/bash
# Round 5: non-temporal vector stores of depth / normals / points (CSG_NT_OUT,
# libcsg_nt.so) vs the production build, at C5 and C3, after the parity file
# through the variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out/r05/ab
CSG_LIB=$PWD/constructionsceneposeestimation_amd/libcsg_nt.so timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r05/ab/pytest_ntout.log 2>&1 || { tail -30 gpurun_out/r05/ab/pytest_ntout.log; exit 1; }
tail -1 gpurun_out/r05/ab/pytest_ntout.log
REPS=3 STEPS=6 FPS=480 EXTRA="--workload C5" SKIP_LDS=1 CTR_VARIANTS="" VARIANTS="base nt" bash tools/gpu_variant_ab.sh || exit 1
mv gpurun_out/r05/ab/tile_ab.txt gpurun_out/r05/ab/ntout_C5.txt
REPS=2 STEPS=6 FPS=2880 SKIP_LDS=1 CTR_VARIANTS="" VARIANTS="base nt" bash tools/gpu_variant_ab.sh || exit 1
mv gpurun_out/r05/ab/tile_ab.txt gpurun_out/r05/ab/ntout_C3.txt
