#!/bin/bash
# Round 5: the plain launcher at the driver's largest N on the box's one GPU:
# `bench.py --gpus 8` starts 8 ranks (sharing the GPU: shared_devices true),
# 240 frames per step each (~10 GB per rank), 4 frames per rank checked.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 900 python3 bench.py --gpus 8 --steps 4 --warmup 1 --frames-per-step 240 --verify-frames-multi 4 > $O/bench_C3_8ranks_plain.json 2> $O/bench_C3_8ranks_plain.err || { tail -20 $O/bench_C3_8ranks_plain.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_C3_8ranks_plain.json')); s=d['shards']; print('8 ranks plain', d['n_gpus'], d['value'], s['disjoint'], s['union'], s['distinct_devices'], s['shared_devices'], d['verified'])"
