#!/bin/bash
# End-to-end generator runs into RAM: the reference's file set (with the point
# cloud) and the set without it; then the file-encoder bench without the point cloud.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/gen_bench.py --frames 240 --batch 30 --writers 16 --dir /dev/shm --outputs reference > gpurun_out/gen_ref.json 2> gpurun_out/gen_ref.err &&
timeout -k 10 300 python tools/gen_bench.py --frames 960 --batch 60 --writers 16 --dir /dev/shm --outputs rgb,mask,depth_csv,depth_png > gpurun_out/gen_nopcd.json 2> gpurun_out/gen_nopcd.err &&
timeout -k 10 200 python tools/files_bench.py --batch 30 --batches 6 --kinds rgb_png,depth_csv,depth_png > gpurun_out/files_bench_3kinds.json 2> gpurun_out/files_bench_3kinds.err
rc=$?
cat gpurun_out/gen_ref.json gpurun_out/gen_nopcd.json gpurun_out/files_bench_3kinds.json; tail -3 gpurun_out/gen_ref.err
exit $rc
