#!/bin/bash
# Round 5: the largest frames (banded binning) and the C3 / C5 lines after the change.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05/maxframe
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_max_frame.py tests/test_gpu_parity.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for w in C3 C5; do
  timeout -k 10 300 python3 bench.py --workload $w --pcie-steps 0 --stats-steps 0 --cpu-single-frames 1 > $O/bench_$w.json 2> $O/bench_$w.err || { tail -5 $O/bench_$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$w.json')); print('$w', d['value'], d['stage_ms_per_step'], d['verified']['bit_exact'])"
done
