#!/bin/bash
# Round 6: k_setup A/B -- the per-(frame, chunk) grid (libcsg.so) against the
# chunk-cull kernel + persistent slot walk (libcsg_sl.so, -DCSG_SETUP_LIST=1),
# 3 runs each in turn, every line self-verified on 32 frames; first the
# ablation build's empty-grid (32) and cull-all (64) settings at the same launch
# size, for the dispatch and cull cost of the grid.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r06/setup_ab
mkdir -p $O
P=constructionsceneposeestimation_amd
for d in ${DBGS-0 32 64}; do
  CSG_LIB=$PWD/$P/libcsg_abl.so CSG_DEBUG=$d timeout -k 10 300 python3 bench.py --verify-frames 0 --steps 5 --pcie-steps 0 --stats-steps 0 > $O/abl_$d.json 2> $O/abl_$d.err || { tail -5 $O/abl_$d.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/abl_$d.json')); print('CSG_DEBUG=$d', d['value'], d['stage_ms_per_step'])" || exit 1
done
for k in 1 2 3; do
  for v in base sl; do
    lib=$PWD/$P/libcsg.so; [ $v = sl ] && lib=$PWD/$P/libcsg_sl.so
    CSG_LIB=$lib timeout -k 10 300 python3 bench.py --pcie-steps 0 --stats-steps 0 > $O/${v}_$k.json 2> $O/${v}_$k.err || { tail -5 $O/${v}_$k.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${v}_$k.json')); print('$v', d['value'], d['stage_ms_per_step'], d['verified']['frames'], d['verified']['bit_exact'])" || exit 1
  done
done
