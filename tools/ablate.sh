#!/bin/bash
# k_raster ablations (CSG_DEBUG bits): 1 no resolve, 2 no raster loop, 4 no alpha test, 256 no level 1,
# 8 no level-2 fragments, 16 no early-z read, 4096 no resolve texture, 8192 no resolve triangle setup,
# 16384 no label stats, 512 profiling counters.  The bits are compiled out of the production
# library (CSG_ABLATION=0); run `tools/build_variant.sh abl - -DCSG_ABLATION=1` first: this script
# loads libcsg_abl.so, one process per setting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export CSG_LIB=${CSG_LIB:-$PWD/constructionsceneposeestimation_amd/libcsg_abl.so}
for d in ${DBGS:-0 1 2 4 8 16 0}; do
  CSG_DEBUG=$d timeout -k 10 200 python bench.py --verify-frames 0 --steps 20 > gpurun_out/ablate_$d.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ablate_$d.json')); print('CSG_DEBUG=$d', d['value'], d['stage_ms_per_step'])"
done
