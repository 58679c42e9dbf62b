#!/bin/bash
# Round 5: non-temporal RGB stores (CSG_NT_RGB, libcsg_ntrgb.so) vs the production
# build (non-temporal depth / normals / points), at C3 and C5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out/r05/ab
CSG_LIB=$PWD/constructionsceneposeestimation_amd/libcsg_ntrgb.so timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_headline.py > gpurun_out/r05/ab/pytest_ntrgb.log 2>&1 || { tail -30 gpurun_out/r05/ab/pytest_ntrgb.log; exit 1; }
tail -1 gpurun_out/r05/ab/pytest_ntrgb.log
REPS=3 STEPS=6 FPS=2880 SKIP_LDS=1 CTR_VARIANTS="" VARIANTS="base ntrgb" bash tools/gpu_variant_ab.sh || exit 1
mv gpurun_out/r05/ab/tile_ab.txt gpurun_out/r05/ab/ntrgb_C3.txt
REPS=2 STEPS=6 FPS=480 EXTRA="--workload C5" SKIP_LDS=1 CTR_VARIANTS="" VARIANTS="base ntrgb" bash tools/gpu_variant_ab.sh || exit 1
mv gpurun_out/r05/ab/tile_ab.txt gpurun_out/r05/ab/ntrgb_C5.txt
