#!/bin/bash
# Round 4 (late): the GPU suite, smoke, the default bench line with its
# kernel-trace profile, C3 at 960 frames per step (the work-memory figure) and
# the other workloads, all with the pooled work buffers.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04
mkdir -p $O
TEST=1 PROF=1 BENCH_ARGS="" bash profiles/r04/tools/gpu_r04_main.sh || exit 1
timeout -k 10 600 python bench.py --frames-per-step 960 --pcie-steps 0 --stats-steps 0 --verify-frames 8 > $O/bench_C3_960.json 2> $O/bench_C3_960.err || { tail -5 $O/bench_C3_960.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_C3_960.json')); print('C3@960', d['value'], d['work']['bytes'], d['verified']['bit_exact'])" || exit 1
WORKLOADS="C2 C4 C5" bash profiles/r04/tools/gpu_r04_configs.sh
