#!/bin/bash
# End of a round: GPU suite + smoke, the default bench line, its kernel-trace
# profile, the PMC passes (HBM traffic, VALU, LDS) at the default launch size,
# the driver's exact command, and the other workloads' lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/final}
mkdir -p $O
export TMPDIR=/tmp
if [ "${TEST:-1}" = 1 ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 600 python3 bench.py > $O/bench_C3.json 2> $O/bench_C3.err || { tail -8 $O/bench_C3.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_C3.json')); print('C3', d['value'], d['roofline']['frac'], d['stage_ms_per_step'], d['verified']['bit_exact'], d['cpu_baseline']['value'])" || exit 1
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_C3_driver.json 2> $O/bench_C3_driver.err || { tail -8 $O/bench_C3_driver.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_C3_driver.json')); print('driver', d['value'], d['roofline']['frac'])" || exit 1
fi
if [ "${PROF:-1}" = 1 ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o kt --output-format csv -- python3 bench.py --verify-frames 0 --pcie-steps 0 --stats-steps 0 > $O/prof_bench.json 2> $O/prof_bench.err || { tail -5 $O/prof_bench.err; exit 1; }
  python3 tools/kernel_stats_by_grid.py $(ls $O/prof/*/kt_kernel_trace.csv $O/prof/kt_kernel_trace.csv 2>/dev/null | head -1) | tee $O/kernel_stats_by_grid.txt
fi
if [ -n "$PMC" ]; then
  ROUND=${ROUND:-final} PASSES="$PMC" bash tools/pmc_profile.sh > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
  tail -3 $O/pmc.log
fi
for w in ${WORKLOADS-C2 C4 C5}; do
  timeout -k 10 600 python3 bench.py --workload $w --pcie-steps 0 --stats-steps 0 > $O/bench_$w.json 2> $O/bench_$w.err || { echo "$w failed"; tail -5 $O/bench_$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$w.json')); print('$w', d['value'], d['roofline']['frac'], d['config']['frames_per_step'], d['verified']['frames'])"
done
