#!/bin/bash
# One A/B session: timing of library variants (LIBS), optional profiling
# counters of ablation builds (CTRS), optional parity tests of one variant (PARITY).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
P=$PWD/constructionsceneposeestimation_amd
for c in ${CTRS}; do
  CSG_LIB=$P/libcsg_$c.so CSG_DEBUG=512 timeout -k 10 200 python bench.py --steps 1 --warmup 0 --verify-frames 0 --pcie-steps 0 --stats-steps 0 ${BENCH_ARGS} > gpurun_out/ctr_$c.json 2> gpurun_out/ctr_$c.err || { echo "ctr $c FAILED"; tail -5 gpurun_out/ctr_$c.err; exit 1; }
  echo "ctr $c: $(grep '\[csg\]' gpurun_out/ctr_$c.err | tail -1)"
done
if [ -n "${PARITY}" ]; then
  CSG_LIB=$P/libcsg_${PARITY}.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/parity_${PARITY}.log 2>&1 || { echo "parity ${PARITY} FAILED"; tail -30 gpurun_out/parity_${PARITY}.log; exit 1; }
  echo "parity ${PARITY}: $(tail -1 gpurun_out/parity_${PARITY}.log)"
fi
LIBS="${LIBS}" REPS=${REPS:-2} bash tools/ab_lib.sh
