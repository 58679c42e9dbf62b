#!/bin/bash
# A/B of the occlusion leg (k_raster<true>): bench's with_occlusion_and_depth_png rate and stage times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
for v in ${LIBS}; do
  CSG_LIB=$PWD/constructionsceneposeestimation_amd/libcsg_$v.so timeout -k 10 200 python bench.py --verify-frames 0 --pcie-steps 0 --stats-steps 5 --steps 10 > gpurun_out/abcov.json 2>gpurun_out/abcov.err || { echo "$v FAILED"; tail -5 gpurun_out/abcov.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/abcov.json')); print('$v', d['value'], d['with_label_stats']['with_occlusion_and_depth_png']['value'])"
done
done
