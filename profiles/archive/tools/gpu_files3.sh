#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_files.py tests/test_gpu_shim.py tests/test_gpu_multirank.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_files.log 2>&1 &&
(export TMPDIR=/tmp; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_files -o kt --output-format csv -- python3 tools/files_bench.py --batch 30 --batches 6 > gpurun_out/files_bench_prof.json 2>&1) &&
timeout -k 10 300 python tools/gen_bench.py --frames 240 --batch 30 --writers 16 --dir /dev/shm --outputs reference > gpurun_out/gen_ref4.json 2> gpurun_out/gen_ref4.err &&
timeout -k 10 300 python tools/gen_bench.py --frames 960 --batch 60 --writers 16 --dir /dev/shm --outputs rgb,mask,depth_csv,depth_png > gpurun_out/gen_nopcd4.json 2> gpurun_out/gen_nopcd4.err
rc=$?
tail -3 gpurun_out/pytest_files.log; cat gpurun_out/gen_ref4.json gpurun_out/gen_nopcd4.json
exit $rc
