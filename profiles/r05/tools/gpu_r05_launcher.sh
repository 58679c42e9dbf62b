#!/bin/bash
# Round 5: the bench's own N-rank launcher on the box (plain `bench.py --gpus 2`,
# no torchrun), the torchrun path beside it, then the default bench line at HEAD.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 880 --timeout-method thread tests/test_gpu_bench_multirank.py > $O/pytest_multirank.log 2>&1 || { tail -30 $O/pytest_multirank.log; exit 1; }
tail -5 $O/pytest_multirank.log
timeout -k 10 600 python3 bench.py --gpus 2 --steps 3 --warmup 1 --frames-per-step 960 --verify-frames-multi 4 > $O/bench_C3_2ranks_plain.json 2> $O/bench_C3_2ranks_plain.err || { tail -20 $O/bench_C3_2ranks_plain.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_C3_2ranks_plain.json')); print('2 ranks plain', d['n_gpus'], d['value'], d['shards'])" || exit 1
timeout -k 10 600 python3 bench.py > $O/bench_C3_start.json 2> $O/bench_C3_start.err || { tail -20 $O/bench_C3_start.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_C3_start.json')); print('C3', d['value'], d['stage_ms_per_step'], d['verified'])"
