#!/bin/bash
# Frames per step (= per launch chain) sweep of the headline bench, production library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/fps_sweep.txt; : > $out
for rep in 1 2; do
for f in ${FS:-240 480 960}; do
  st=$((${TOTAL:-4800} / f))
  timeout -k 10 300 python bench.py --verify-frames 0 --pcie-steps 0 --stats-steps 0 --frames-per-step $f --steps $st > gpurun_out/fps.json 2> gpurun_out/fps.err || { echo "F=$f FAILED" >> $out; tail -5 gpurun_out/fps.err >> $out; cat $out; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/fps.json')); print('F=$f steps=$st', d['value'], d['stage_ms_per_step'])" >> $out
  echo "rep $rep F=$f done"
done
done
cat $out
