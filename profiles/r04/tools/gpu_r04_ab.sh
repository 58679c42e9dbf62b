#!/bin/bash
# Round 4: (optional) exhaustive reciprocal check, the GPU suite on the working
# tree's library, then an A/B of library variants (LIBS, built by
# tools/build_variant.sh) at the bench's default launch size.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04
mkdir -p $O
if [ -n "$RCP" ]; then
  # the proven range |x| in [2^-126, 2^126] of each sign, then the rest of the normals
  timeout -k 10 120 ./tools/rcp_check 0x00800000 0x7E800001 > $O/rcp_pos_range.json &&
  timeout -k 10 120 ./tools/rcp_check 0x80800000 0xFE800001 > $O/rcp_neg_range.json &&
  timeout -k 10 120 ./tools/rcp_check 0x7E800001 0x7F800000 > $O/rcp_pos_top.json &&
  timeout -k 10 120 ./tools/rcp_check 0xFE800001 0xFF800000 > $O/rcp_neg_top.json || exit 1
  cat $O/rcp_pos_range.json $O/rcp_neg_range.json $O/rcp_pos_top.json $O/rcp_neg_top.json
fi
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; tail -3 $O/pytest_gpu.log; grep -A30 "FAIL\|Error" $O/pytest_gpu.log | head -40
  [ $rc -ne 0 ] && exit $rc
fi
LIBS="${LIBS:-base cur}" REPS=${REPS:-3} STEPS=${STEPS:-6} bash tools/ab_lib.sh 2>&1 | tee $O/ab.txt
