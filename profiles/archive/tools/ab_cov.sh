#!/bin/bash
# A/B timing of the occlusion + depth PNG leg (bench.py with_label_stats):
#   LIBS="base cov" bash tools/ab_cov.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
for v in ${LIBS}; do
  CSG_LIB=$PWD/constructionsceneposeestimation_amd/libcsg_$v.so timeout -k 10 200 python bench.py --verify-frames 0 --pcie-steps 0 --stats-steps ${STATS:-10} --steps ${STEPS:-10} > gpurun_out/abcov.json 2>gpurun_out/abcov.err || { echo "$v FAILED"; tail -5 gpurun_out/abcov.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/abcov.json')); s=d['with_label_stats']; print('$v', d['value'], s['value'], s['with_occlusion_and_depth_png']['value'])"
done
done
