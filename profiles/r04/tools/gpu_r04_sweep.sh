#!/bin/bash
# Round 4: launch-size sweep with sized work buffers (C3 frames per step, C5
# frames per step) and the generator with occlusion coverage off / on.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04
mkdir -p $O
quick="--verify-frames 0 --pcie-steps 0 --stats-steps 0"
line() { python3 -c "import json,sys; d=json.load(open('$1')); print('$2', d['value'], d['ms_per_step'], 'work_GB', round(d['work']['bytes']/1e9,2), d['stage_ms_per_step'])"; }
for rep in 1 2; do
  for F in ${C3_STEPS:-960 1920 2880 3840}; do
    K=$((19200 / F))
    timeout -k 10 300 python bench.py --frames-per-step $F --steps $K --warmup 2 $quick > $O/c3_$F.$rep.json 2> $O/c3_$F.$rep.err || { echo "C3 F=$F failed"; tail -5 $O/c3_$F.$rep.err; exit 1; }
    line $O/c3_$F.$rep.json "C3 F=$F rep=$rep" | tee -a $O/sweep.txt
  done
done
for F in ${C5_STEPS:-240 480}; do
  K=$((2400 / F))
  timeout -k 10 300 python bench.py --workload C5 --frames-per-step $F --steps $K --warmup 1 $quick > $O/c5_$F.json 2> $O/c5_$F.err || { echo "C5 F=$F failed"; tail -5 $O/c5_$F.err; exit 1; }
  line $O/c5_$F.json "C5 F=$F" | tee -a $O/sweep.txt
done
if [ -n "$GEN" ]; then
  for occ in "" "--occlusion"; do
    timeout -k 10 400 python tools/gen_bench.py --frames 480 --batch 60 --writers 16 --outputs rgb,mask,depth_csv,depth_png --dir /dev/shm --skip-extras $occ > $O/gen$occ.json 2> $O/gen$occ.err || { echo "gen $occ failed"; tail -5 $O/gen$occ.err; exit 1; }
    cat $O/gen$occ.json | tee -a $O/sweep.txt
  done
fi
