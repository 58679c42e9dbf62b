#!/bin/bash
# Round 4: bench lines of the other workloads at the default launch sizes, and
# the CPU-baseline thread scaling (box CPUs, 16-CPU share).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04
mkdir -p $O
for w in ${WORKLOADS:-C2 C4 C5}; do
  timeout -k 10 600 python bench.py --workload $w --pcie-steps 0 --stats-steps 0 > $O/bench_$w.json 2> $O/bench_$w.err || { echo "$w failed"; tail -5 $O/bench_$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$w.json')); print('$w', d['value'], d['roofline']['frac'], d['config']['frames_per_step'], d['work']['bytes'], d['verified']['frames'], d['cpu_baseline']['value'])"
done
if [ -n "$CPU" ]; then
  timeout -k 10 400 python tools/cpu_scaling.py > $O/cpu_scaling.json 2> $O/cpu_scaling.err || { tail -5 $O/cpu_scaling.err; exit 1; }
  cat $O/cpu_scaling.json
fi
