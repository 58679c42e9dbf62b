#!/bin/bash
# A/B: compiler options for the whole library: the AMDGPU scheduler's own
# register-pressure trackers (trk), -O2 (o2), vs HEAD at -O3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PARITY=trk LIBS="base trk o2" REPS=3 bash tools/ab_round.sh 2>&1 | tee gpurun_out/ab_flags.txt
