#!/bin/bash
# Round-2 ablation split of k_raster on the spec-fidelity C3 workload: time per
# CSG_DEBUG setting (libcsg_abl.so) plus the profiling counters (CSG_DEBUG=512).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export CSG_LIB=$PWD/constructionsceneposeestimation_amd/libcsg_abl.so
CSG_DEBUG=512 timeout -k 10 200 python bench.py --steps 1 --warmup 0 --verify-frames 0 --pcie-steps 0 --stats-steps 0 > gpurun_out/ctr.json 2> gpurun_out/ctr.err || exit 1
grep "\[csg\]" gpurun_out/ctr.err | tail -1
DBGS="${DBGS:-0 1 2 4 8 16 256 4096 8192 1024}" bash tools/ablate.sh
