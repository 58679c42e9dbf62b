#!/bin/bash
# Round 5: the GPU suite (all -m gpu tests, one process), then the launcher's
# plain N=2 run at 960 frames per step and the default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
if [ "${BENCH:-1}" = 1 ]; then
timeout -k 10 600 python3 bench.py --gpus 2 --steps 3 --warmup 1 --frames-per-step 960 --verify-frames-multi 4 > $O/bench_C3_2ranks_plain.json 2> $O/bench_C3_2ranks_plain.err || { tail -20 $O/bench_C3_2ranks_plain.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_C3_2ranks_plain.json')); print('2 ranks plain', d['n_gpus'], d['value'], d['shards']['devices'], d['shards']['shared_devices'])" || exit 1
timeout -k 10 600 python3 bench.py > $O/bench_C3_start.json 2> $O/bench_C3_start.err || { tail -20 $O/bench_C3_start.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_C3_start.json')); print('C3', d['value'], d['stage_ms_per_step'], d['verified'], d['work']['hint_retries'] if 'hint_retries' in d['work'] else '')"
fi
