#!/bin/bash
# Round 5: GPU suite + bench with the per-chain host copies (copy stream), then
# the level-1 edge precompute (CSG_L1_PRE) on the 32x16 build: parity tests
# through it and an A/B at the bench's launch size.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TEST=1 BENCH=1 PROF=0 WORKLOADS="" bash tools/gpu_final.sh || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r05/final/bench_C3.json')); print('pcie', d['pcie_inclusive'])"
L=$PWD/constructionsceneposeestimation_amd
mkdir -p gpurun_out/r05
CSG_LIB=$L/libcsg_l1pre.so timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_lds_order.py tests/test_gpu_headline.py > gpurun_out/r05/pytest_l1pre.log 2>&1 || { tail -30 gpurun_out/r05/pytest_l1pre.log; exit 1; }
tail -1 gpurun_out/r05/pytest_l1pre.log
REPS=${REPS:-2} STEPS=6 FPS=2880 SKIP_LDS=1 CTR_VARIANTS="" VARIANTS="base l1pre" bash tools/gpu_variant_ab.sh
