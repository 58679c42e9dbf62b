#!/bin/bash
# Round 5: the generator at steady state (>= 20,000 frames, files to /dev/null,
# with and without the point cloud; 2,000 frames into /dev/shm without it) and
# the CPU baseline's thread scaling with the box's CPU share recorded.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05/gen
mkdir -p $O
N=${FRAMES:-20000}
NO_PC=rgb,mask,depth_csv,depth_png
timeout -k 10 400 python3 -u tools/gen_steady.py --frames $N --outputs reference --sink discard > $O/steady_reference.json 2> $O/steady_reference.err || { tail -20 $O/steady_reference.err; exit 1; }
cat $O/steady_reference.json
timeout -k 10 300 python3 -u tools/gen_steady.py --frames $N --outputs $NO_PC --sink discard > $O/steady_no_pointcloud.json 2> $O/steady_no_pointcloud.err || { tail -20 $O/steady_no_pointcloud.err; exit 1; }
cat $O/steady_no_pointcloud.json
timeout -k 10 300 python3 -u tools/gen_steady.py --frames ${SHM_FRAMES:-2000} --outputs $NO_PC --sink disk --dir /dev/shm > $O/shm_no_pointcloud.json 2> $O/shm_no_pointcloud.err || { tail -20 $O/shm_no_pointcloud.err; exit 1; }
cat $O/shm_no_pointcloud.json
if [ "${CPU:-1}" = 1 ]; then
timeout -k 10 300 python3 -u tools/cpu_scaling.py --frames 32 > $O/cpu_scaling.json 2> $O/cpu_scaling.err || { tail -5 $O/cpu_scaling.err; exit 1; }
cat $O/cpu_scaling.json
fi
