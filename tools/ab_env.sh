#!/bin/bash
# A/B of an environment knob on bench.py: ENVS="CSG_BINBLOCKS=32 CSG_BINBLOCKS=128" bash tools/ab_env.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for e in ${ENVS}; do
  env $e timeout -k 10 200 python bench.py --cpu-sample 0 --steps 20 > gpurun_out/abenv.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/abenv.json')); print('$e', d['value'], d['stage_ms_per_step'])"
done
