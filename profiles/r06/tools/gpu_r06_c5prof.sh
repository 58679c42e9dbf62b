#!/bin/bash
# Round 6: rocprofv3 kernel trace of the C5 (3840x2160, depth + normals + points)
# and C2 bench lines, summarised per kernel and grid.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r06/wprof
mkdir -p $O
for w in C5 C2; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/$w -o kt --output-format csv -- python3 bench.py --workload $w --verify-frames 0 --pcie-steps 0 --stats-steps 0 > $O/bench_$w.json 2> $O/bench_$w.err || { tail -5 $O/bench_$w.err; exit 1; }
  python3 tools/kernel_stats_by_grid.py $(ls $O/$w/*/kt_kernel_trace.csv $O/$w/kt_kernel_trace.csv 2>/dev/null | head -1) > $O/kernel_stats_by_grid_$w.txt || exit 1
  head -12 $O/kernel_stats_by_grid_$w.txt
done
