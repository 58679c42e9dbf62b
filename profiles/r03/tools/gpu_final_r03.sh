#!/bin/bash
# Round-3 closing evidence at the default bench configuration: smoke, GPU suite,
# bench line, rocprofv3 kernel stats (tools/gpu_check.sh), then the PMC traffic
# and VALU passes that feed bench.py's roofline.traffic / valu (profiles/pmc_traffic.json).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROUND=r03 bash tools/gpu_check.sh &&
ROUND=r03f PASSES="fetch write valu" BENCH_ARGS="--steps 4 --warmup 1 --verify-frames 0 --pcie-steps 0 --stats-steps 0" bash tools/pmc_profile.sh > gpurun_out/pmc_r03f.txt 2>&1 &&
python3 tools/pmc_summarize.py gpurun_out/pmc_r03f --write-profile > /dev/null &&
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
