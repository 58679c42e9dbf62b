#!/bin/bash
# Closing bench lines of the other configurations (C2, C4, C5) at HEAD.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cfg
for w in C2 C4 C5; do
  timeout -k 10 400 python bench.py --workload $w > gpurun_out/cfg/bench_$w.json 2> gpurun_out/cfg/bench_$w.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/cfg/bench_$w.json')); print('$w', d['value'], d['roofline']['frac'], d['verified']['bit_exact'], d['cpu_baseline']['value'])"
done
