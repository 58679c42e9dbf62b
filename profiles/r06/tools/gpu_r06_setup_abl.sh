#!/bin/bash
# Round 6: where k_setup's time goes (ablation build, CSG_DEBUG bits): all work,
# stop after the frustum test (0x10000: loads + transform + frustum test of every
# triangle of a surviving chunk), cull all (64), empty grid (32); 2 runs each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r06/setup_abl
mkdir -p $O
for k in 1 2; do
  for d in 0 65536 64 32; do
    CSG_LIB=$PWD/constructionsceneposeestimation_amd/libcsg_abl.so CSG_DEBUG=$d timeout -k 10 300 python3 bench.py --verify-frames 0 --steps 5 --pcie-steps 0 --stats-steps 0 > $O/abl_${d}_$k.json 2> $O/abl_${d}_$k.err || { tail -5 $O/abl_${d}_$k.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/abl_${d}_$k.json')); print('CSG_DEBUG=$d', d['stage_ms_per_step'])" || exit 1
  done
done
