#!/bin/bash
# Round 4 (end): the GPU suite and smoke, the default bench line with its
# kernel-trace profile, the driver's exact command, C2/C4/C5 lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04
mkdir -p $O
TEST=1 PROF=1 BENCH_ARGS="" bash profiles/r04/tools/gpu_r04_main.sh || exit 1
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -5 $O/bench_driver.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_driver.json')); print('driver', d['value'], d['work']['bytes'], d['verified']['bit_exact'])" || exit 1
WORKLOADS="C2 C4 C5" bash profiles/r04/tools/gpu_r04_configs.sh
