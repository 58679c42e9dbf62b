#!/bin/bash
# Round 5: a vector group's shading loop skips the depth (CSG_VEC_DEP_ONCE,
# libcsg_deponce.so) -- parity through it, then C5 against production.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out/r05/ab
CSG_LIB=$PWD/constructionsceneposeestimation_amd/libcsg_deponce.so timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_lds_order.py > gpurun_out/r05/ab/pytest_deponce.log 2>&1 || { tail -30 gpurun_out/r05/ab/pytest_deponce.log; exit 1; }
tail -1 gpurun_out/r05/ab/pytest_deponce.log
REPS=3 STEPS=6 FPS=480 EXTRA="--workload C5" SKIP_LDS=1 CTR_VARIANTS="" VARIANTS="base deponce" bash tools/gpu_variant_ab.sh || exit 1
mv gpurun_out/r05/ab/tile_ab.txt gpurun_out/r05/ab/deponce_C5.txt
