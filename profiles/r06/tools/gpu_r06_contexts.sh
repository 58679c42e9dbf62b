#!/bin/bash
# Round 6: two renderer contexts (alternate steps on their own streams, so one
# step's k_setup / binning can start under the other's k_raster tail) against
# one, at the bench's 2,880 frames per step; 2 runs each in turn, verified.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r06/contexts
mkdir -p $O
for k in 1 2; do
  for n in 1 2; do
    timeout -k 10 400 python3 bench.py --contexts $n --pcie-steps 0 --stats-steps 0 > $O/ctx${n}_$k.json 2> $O/ctx${n}_$k.err || { tail -5 $O/ctx${n}_$k.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/ctx${n}_$k.json')); print('contexts $n', d['value'], d['ms_per_step'], d['stage_ms_per_step'], d['verified']['bit_exact'])" || exit 1
  done
done
