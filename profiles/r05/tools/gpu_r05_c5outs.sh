#!/bin/bash
# Round 5: C5's per-pixel outputs' share of k_raster (profiles/r05/tools/c5_outputs_probe.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r05/c5outs
mkdir -p $O
for rep in 1 2; do
for outs in rgb,instance,keypoints rgb,instance,depth,keypoints rgb,instance,depth,normals,keypoints rgb,instance,depth,points,keypoints rgb,instance,depth,normals,points,keypoints; do
  timeout -k 10 300 python3 profiles/r05/tools/c5_outputs_probe.py $outs --pcie-steps 0 --stats-steps 0 --cpu-single-frames 1 --verify-frames 8 > $O/c5_$outs.json 2> $O/c5_$outs.err || { tail -5 $O/c5_$outs.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c5_$outs.json')); print('$outs rep $rep', d['value'], d['stage_ms_per_step'], d['verified']['bit_exact'])" | tee -a $O/c5_outputs.txt
done
done
