#!/bin/bash
# Bench lines of the other configurations (C2, C4, C5) and PMC passes of the
# file encoders (files_bench): FETCH_SIZE, WRITE_SIZE, VALU busy.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cfg gpurun_out/pmc_files
export TMPDIR=/tmp
rc=0
for w in C2 C4 C5; do
  timeout -k 10 400 python bench.py --workload $w > gpurun_out/cfg/bench_$w.json 2> gpurun_out/cfg/bench_$w.err || { rc=$?; break; }
done
if [ $rc -eq 0 ]; then
  for p in "fetch FETCH_SIZE" "write WRITE_SIZE" "valu SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"; do
    set -- $p; name=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc_files/$name -o pmc -- python3 tools/files_bench.py --batch 30 --batches 3 > gpurun_out/pmc_files/$name.json 2> gpurun_out/pmc_files/$name.err || { rc=$?; break; }
  done
fi
if [ $rc -eq 0 ]; then
  ROUND=r03 PASSES="fetch write" bash tools/pmc_profile.sh > gpurun_out/pmc_r03_traffic.txt 2>&1 || rc=$?
fi
for w in C2 C4 C5; do python3 -c "import json; d=json.load(open('gpurun_out/cfg/bench_$w.json')); print('$w', d['value'], d['cpu_baseline'])" 2>/dev/null; done
exit $rc
