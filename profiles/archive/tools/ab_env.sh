#!/bin/bash
# A/B of environment knobs on bench.py; one entry per run, knobs joined by ':'
#   ENVS="CSG_CHAIN=60:CSG_TILEMAP=0 CSG_CHAIN=8:CSG_TILEMAP=1" bash tools/ab_env.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
REPS=${REPS:-1}
for rep in $(seq $REPS); do
for e in ${ENVS}; do
  env ${e//:/ } timeout -k 10 200 python bench.py --verify-frames 0 --steps ${STEPS:-20} ${BENCH_ARGS} > gpurun_out/abenv.json 2>/dev/null || { echo "$e FAILED"; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/abenv.json')); print('$e', d['value'], d['stage_ms_per_step'], d['roofline']['avg_launch_ms'])"
done
done
