#!/bin/bash
# Round 4: exhaustive reciprocal check, the default bench line, its
# kernel-trace profile and the PMC passes at the default launch size.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04
mkdir -p $O
export TMPDIR=/tmp
if [ -n "$RCP" ]; then
  timeout -k 10 120 ./tools/rcp_check > $O/rcp_pos.json &&
  timeout -k 10 120 ./tools/rcp_check 0x80800000 0xFF800000 > $O/rcp_neg.json || exit 1
  cat $O/rcp_pos.json $O/rcp_neg.json
fi
if [ -n "$TEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; tail -3 $O/pytest_gpu.log; grep -A30 "FAIL\|Error" $O/pytest_gpu.log | head -40
  [ $rc -ne 0 ] && exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
fi
timeout -k 10 600 python bench.py $BENCH_ARGS > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d['work']['bytes'], d['stage_ms_per_step'])"
if [ -n "$PROF" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o kt --output-format csv -- python3 bench.py --verify-frames 0 --pcie-steps 0 --stats-steps 0 $BENCH_ARGS > $O/prof_bench.json 2> $O/prof_bench.err || exit 1
  python3 tools/kernel_stats_by_grid.py $(ls $O/prof/*/kt_kernel_trace.csv $O/prof/kt_kernel_trace.csv 2>/dev/null | head -1) | tee $O/kernel_stats_by_grid.txt
fi
if [ -n "$PMC" ]; then
  ROUND=r04 PASSES="$PMC" bash tools/pmc_profile.sh > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
  tail -3 $O/pmc.log
fi
