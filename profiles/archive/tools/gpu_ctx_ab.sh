#!/bin/bash
# A/B of renderer contexts per GPU in bench.py (--contexts 1 vs 2 vs 3), then a
# verified --contexts 2 line.  Timing probes: verify off in the A/B loop.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/ctx_ab.txt
: > $out
for rep in $(seq ${REPS:-3}); do
for n in ${CTXS:-1 2 3}; do
  timeout -k 10 200 python bench.py --verify-frames 0 --pcie-steps 0 --stats-steps 0 --steps ${STEPS:-20} \
      --contexts $n ${BENCH_ARGS} > gpurun_out/ctx.json 2>gpurun_out/ctx.err || { echo "ctx $n FAILED" >> $out; tail -5 gpurun_out/ctx.err >> $out; cat $out; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ctx.json')); print('ctx $n', d['value'], d['stage_ms_per_step'])" >> $out
  echo "rep $rep ctx $n done"
done
done
timeout -k 10 300 python bench.py --contexts 2 ${BENCH_ARGS} > gpurun_out/bench_ctx2.json 2>gpurun_out/bench_ctx2.err || { echo "verified ctx2 FAILED" >> $out; tail -8 gpurun_out/bench_ctx2.err >> $out; cat $out; exit 1; }
cat $out
cat gpurun_out/bench_ctx2.json
