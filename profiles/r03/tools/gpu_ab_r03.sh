#!/bin/bash
# GPU suite on the working tree's library, then A/B of library variants (LIBS).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
LIBS="${LIBS:-base cur}" REPS=${REPS:-2} bash tools/ab_lib.sh > gpurun_out/ab.txt 2>&1
rc=$?
tail -4 gpurun_out/pytest_gpu.log; grep -B2 -A20 "FAIL\|Error" gpurun_out/pytest_gpu.log | head -60; cat gpurun_out/ab.txt
exit $rc
