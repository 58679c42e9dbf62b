#!/bin/bash
# Round 5: the swizzled z-buffer (CSG_ZB_SWIZZLE) -- parity subset, A/B against
# the row-major layout at 32x32 and 32x16 tiles, LDS counters of the new layout.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_lds_order.py tests/test_gpu_keypoint_sky.py tests/test_gpu_occlusion_depthvis.py tests/test_gpu_headline.py > $O/pytest_swz.log 2>&1 || { tail -30 $O/pytest_swz.log; exit 1; }
tail -2 $O/pytest_swz.log
REPS=${REPS:-3} VARIANTS="${VARIANTS:-base noswz w32h16 w32h16_noswz w32h16:CSG_BINBLOCKS=16}" CTR_VARIANTS="" DBGS="${DBGS:-0 1 8}" LDS_TAG=_swz bash tools/gpu_variant_ab.sh
