#!/bin/bash
# Round 4 (late): the pooled work buffers at the driver's bench command, then
# the level-1 edge precompute variant (libcsg_l1.so): parity tests and A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_bench_multirank.py tests/test_gpu_sizing.py -x -v --timeout 600 --timeout-method thread > $O/pytest_bench_tests.log 2>&1
rc=$?; tail -4 $O/pytest_bench_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -5 $O/bench_driver.err; exit 1; }
grep -i "failed" $O/bench_driver.err
python3 -c "import json; d=json.load(open('$O/bench_driver.json')); print('driver', d['value'], d['work']['bytes'], d['verified']['bit_exact'], d['pcie_inclusive']['value'], d['with_label_stats']['value'])" || exit 1
CSG_LIB=$PWD/constructionsceneposeestimation_amd/libcsg_l1.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_keypoint_sky.py tests/test_gpu_occlusion_depthvis.py -x -q --timeout 300 --timeout-method thread > $O/pytest_l1.log 2>&1
rc=$?; tail -3 $O/pytest_l1.log; [ $rc -ne 0 ] && exit $rc
LIBS="cur l1" REPS=3 STEPS=6 bash tools/ab_lib.sh 2>&1 | tee $O/ab_l1.txt
