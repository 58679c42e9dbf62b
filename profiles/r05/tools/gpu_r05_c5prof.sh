#!/bin/bash
# Round 5: rocprofv3 kernel-trace summary of the C5 bench line (final kernels).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r05/c5prof
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o kt --output-format csv -- python3 bench.py --workload C5 --verify-frames 0 --pcie-steps 0 --stats-steps 0 > $O/bench_C5_prof.json 2> $O/bench_C5_prof.err || { tail -5 $O/bench_C5_prof.err; exit 1; }
python3 tools/kernel_stats_by_grid.py $(ls $O/prof/*/kt_kernel_trace.csv $O/prof/kt_kernel_trace.csv 2>/dev/null | head -1) | tee $O/kernel_stats_by_grid_C5.txt
