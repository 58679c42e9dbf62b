#!/bin/bash
# Round-3 evidence for k_raster: ablation split + profiling counters (libcsg_abl.so)
# and the VALU / SQ counter passes of the production library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
DBGS="${DBGS:-0 1 2 4 8 16 256 4096 8192 32 64 128 0}" bash tools/ablate_r02.sh > gpurun_out/ablate_r03.txt 2>&1 &&
ROUND=${PMCR:-r03} PASSES="${PASSES:-sq valu}" bash tools/pmc_profile.sh > gpurun_out/pmc_${PMCR:-r03}.txt 2>&1
rc=$?
cat gpurun_out/ablate_r03.txt; tail -40 gpurun_out/pmc_r03.txt
exit $rc
