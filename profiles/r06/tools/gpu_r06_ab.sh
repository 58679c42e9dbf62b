#!/bin/bash
# Round 6 k_raster A/B: parity tests of the working-tree libcsg.so first
# (TESTS, default the parity files that exercise the raster loop), then
# tools/gpu_variant_ab.sh on bench.py (VARIANTS, REPS, FPS; each line verified
# bit-exact on 8 frames).  Results under $OUT (default gpurun_out/r06/ab).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r06/ab}
mkdir -p $O
if [ "${TESTS-x}" != "" ]; then
  T=${TESTS:-tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_lds_order.py tests/test_gpu_keypoint_sky.py tests/test_gpu_max_frame.py}
  timeout -k 10 900 python3 -u -m pytest $T -x -v --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
OUT=$O VARIANTS="${VARIANTS:-old base}" REPS=${REPS:-3} FPS=${FPS:-2880} STEPS=${STEPS:-6} SKIP_LDS=1 CTR_VARIANTS="" \
  bash tools/gpu_variant_ab.sh || exit 1
