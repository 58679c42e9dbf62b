#!/bin/bash
# One GPU session: smoke, GPU tests, bench, kernel-trace profile.  Every GPU step
# has its own time limit and the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=${ROUND:-r02}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 400 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err &&
(export TMPDIR=/tmp; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$R -o kt --output-format csv -- python3 bench.py --verify-frames 0 --pcie-steps 0 --stats-steps 0 ${BENCH_ARGS} > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err)
rc=$?
echo "exit $rc"
tail -3 gpurun_out/smoke.log; tail -5 gpurun_out/pytest_gpu.log; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
exit $rc
