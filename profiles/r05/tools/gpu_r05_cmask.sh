#!/bin/bash
# Round 5: k_setup's small-cover test as a 16-bit coverage mask (CSG_COVER_MASK):
# parity through it, then an A/B at the bench's launch size.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=$PWD/constructionsceneposeestimation_amd
mkdir -p gpurun_out/r05
CSG_LIB=$L/libcsg_cmask.so timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_sizing.py > gpurun_out/r05/pytest_cmask.log 2>&1 || { tail -30 gpurun_out/r05/pytest_cmask.log; exit 1; }
tail -1 gpurun_out/r05/pytest_cmask.log
REPS=${REPS:-3} STEPS=6 FPS=2880 SKIP_LDS=1 CTR_VARIANTS="" VARIANTS="base cmask" bash tools/gpu_variant_ab.sh
