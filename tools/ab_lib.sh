#!/bin/bash
# A/B timing of library variants: LIBS="base soa" bash tools/ab_lib.sh
# (constructionsceneposeestimation_amd/libcsg_<name>.so, built by tools/build_variant.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
for v in ${LIBS}; do
  CSG_LIB=$PWD/constructionsceneposeestimation_amd/libcsg_$v.so timeout -k 10 200 python bench.py --verify-frames 0 --pcie-steps 0 --stats-steps 0 --steps ${STEPS:-20} ${BENCH_ARGS} > gpurun_out/ablib.json 2>gpurun_out/ablib.err || { echo "$v FAILED"; tail -5 gpurun_out/ablib.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ablib.json')); print('$v', d['value'], d['stage_ms_per_step'])"
done
done
