#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/gen_bench.py --frames 240 --batch 30 --writers 16 --dir /dev/shm --outputs reference > gpurun_out/gen_ref4.json 2> gpurun_out/gen_ref4.err &&
timeout -k 10 300 python tools/gen_bench.py --frames 960 --batch 60 --writers 16 --dir /dev/shm --outputs rgb,mask,depth_csv,depth_png > gpurun_out/gen_nopcd4.json 2> gpurun_out/gen_nopcd4.err
rc=$?
cat gpurun_out/gen_ref4.json gpurun_out/gen_nopcd4.json; tail -3 gpurun_out/gen_ref4.err
exit $rc
