#!/bin/bash
# Round 6: the generator at steady state with the narrowed instance-id wire
# (20,000 frames, files to /dev/null, without and with the point cloud; 2,000
# frames into /dev/shm without it), and the no-point-cloud run again with the
# int32 wire (CSG_NARROW_IDS=0) on the same box for the A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r06/gen
mkdir -p $O
N=${FRAMES:-20000}
NO_PC=rgb,mask,depth_csv,depth_png
timeout -k 10 300 python3 -u tools/gen_steady.py --frames $N --outputs $NO_PC --sink discard > $O/steady_no_pointcloud.json 2> $O/steady_no_pointcloud.err || { tail -20 $O/steady_no_pointcloud.err; exit 1; }
cat $O/steady_no_pointcloud.json
CSG_NARROW_IDS=0 timeout -k 10 300 python3 -u tools/gen_steady.py --frames $N --outputs $NO_PC --sink discard > $O/steady_no_pointcloud_int32.json 2> $O/steady_no_pointcloud_int32.err || { tail -20 $O/steady_no_pointcloud_int32.err; exit 1; }
cat $O/steady_no_pointcloud_int32.json
timeout -k 10 400 python3 -u tools/gen_steady.py --frames $N --outputs reference --sink discard > $O/steady_reference.json 2> $O/steady_reference.err || { tail -20 $O/steady_reference.err; exit 1; }
cat $O/steady_reference.json
timeout -k 10 300 python3 -u tools/gen_steady.py --frames ${SHM_FRAMES:-2000} --outputs $NO_PC --sink disk --dir /dev/shm > $O/shm_no_pointcloud.json 2> $O/shm_no_pointcloud.err || { tail -20 $O/shm_no_pointcloud.err; exit 1; }
cat $O/shm_no_pointcloud.json
# launch-chain splitting for pageable host outputs, A/B
timeout -k 10 300 python3 -u tools/pageable_ab.py --frames 480 > $O/pageable_ab.json 2> $O/pageable_ab.err || { tail -20 $O/pageable_ab.err; exit 1; }
cat $O/pageable_ab.json
if [ "${N2:-1}" = 1 ]; then
  # the N = 2 line as `bench.py --gpus 2` prints it (two ranks sharing the box's one GPU)
  timeout -k 10 600 python3 bench.py --gpus 2 > $O/bench_C3_n2.json 2> $O/bench_C3_n2.err || { tail -20 $O/bench_C3_n2.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_C3_n2.json')); print('n2', d['value'], d['shards']['per_rank'], d['shards']['imbalance'], d['pcie_inclusive'])"
fi
