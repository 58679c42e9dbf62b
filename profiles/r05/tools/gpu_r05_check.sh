#!/bin/bash
# Round 5: the GPU suite and the default bench line after a kernel change, then
# the per-phase VALU split of the ablation build (tools/gpu_ablate_valu.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TEST=1 BENCH=1 PROF=${PROF:-0} WORKLOADS="" bash tools/gpu_final.sh || exit 1
if [ "${ABL:-1}" = 1 ]; then
  bash tools/gpu_ablate_valu.sh || exit 1
fi
