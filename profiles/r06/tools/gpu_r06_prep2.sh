#!/bin/bash
# Round 6: the no-point-cloud steady state with 2 prep workers, 3 vs 4 renderer
# contexts and batches of 60 vs 120 frames, in turn, on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r06/prep2
mkdir -p $O
NO_PC=rgb,mask,depth_csv,depth_png
for k in 1 2; do
  for cfg in "3 60" "4 60" "3 120"; do
    set -- $cfg
    n=r$1_b$2_$k
    timeout -k 10 300 python3 -u tools/gen_steady.py --frames ${FRAMES:-20000} --outputs $NO_PC --sink discard --prep-workers 2 --renderers $1 --batch $2 > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['frames_per_s'], d['writer_busy'], d['render_busy'], d['render_thread'], d['d2h_gbs'])"
  done
done
