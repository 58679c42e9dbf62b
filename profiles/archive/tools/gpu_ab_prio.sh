#!/bin/bash
# A/B: wave priority raised (s_setprio 2) while k_raster issues its staging loads
# (prio1) and also the resolve's triangle-setup loads (prio3), vs HEAD.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PARITY=prio3 LIBS="base prio0 prio1 prio3" REPS=3 bash tools/ab_round.sh 2>&1 | tee gpurun_out/ab_prio.txt
