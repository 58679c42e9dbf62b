#!/bin/bash
# A/B of library variants only (LIBS), no test suite (timing probes whose outputs may be wrong).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIBS="${LIBS:-base}" REPS=${REPS:-2} bash tools/ab_lib.sh > gpurun_out/ab.txt 2>&1
rc=$?
cat gpurun_out/ab.txt
exit $rc
