#!/bin/bash
# Bench lines of the other configurations at bench.py's defaults (C2, C4, C5).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cfg
for w in ${WLS:-C2 C4 C5}; do
  SECONDS=0
  timeout -k 10 500 python bench.py --workload $w > gpurun_out/cfg/bench_$w.json 2> gpurun_out/cfg/bench_$w.err || { echo "$w FAILED"; tail -5 gpurun_out/cfg/bench_$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/cfg/bench_$w.json')); print('$w', d['value'], d['config']['frames_per_step'], d['roofline']['frac'], d['verified']['bit_exact'], d['cpu_baseline']['value'], '${SECONDS}s')"
done
