#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -k "c4 or two_rank" -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_misc.log 2>&1 &&
timeout -k 10 300 python tools/gen_bench.py --frames 240 --batch 30 --writers 16 --dir /dev/shm --outputs reference > gpurun_out/gen_ref2.json 2> gpurun_out/gen_ref2.err
rc=$?
tail -8 gpurun_out/pytest_misc.log; cat gpurun_out/gen_ref2.json; tail -3 gpurun_out/gen_ref2.err
exit $rc
