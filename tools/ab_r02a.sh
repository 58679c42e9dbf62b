#!/bin/bash
# round-2 A/B: mask records + level-1 class order (mask), + coarse z (full), vs the previous kernels (base)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
LIBS="base mask full" REPS=2 timeout -k 10 600 bash tools/ab_lib.sh || exit 1
for v in ablbase abl; do
  CSG_LIB=$PWD/constructionsceneposeestimation_amd/libcsg_$v.so CSG_DEBUG=512 timeout -k 10 200 python bench.py --steps 1 --warmup 0 --verify-frames 0 --pcie-steps 0 --stats-steps 0 > gpurun_out/ctr_$v.json 2> gpurun_out/ctr_$v.err || exit 1
  echo $v; grep "\[csg\]" gpurun_out/ctr_$v.err | tail -1
done
