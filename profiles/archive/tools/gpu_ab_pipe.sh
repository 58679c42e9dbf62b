#!/bin/bash
# A/B: level-2 rank query of the next item issued before the current fragment
# (pipe), plus the early-z word read at the top of the fragment (pipez), vs HEAD.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PARITY=pipez LIBS="base pipe pipez" REPS=3 bash tools/ab_round.sh 2>&1 | tee gpurun_out/ab_pipe.txt
