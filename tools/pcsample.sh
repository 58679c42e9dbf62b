#!/bin/bash
# PC sampling of bench.py (k_raster hot spots).  rocprofv3 -L first (lists the
# PC-sampling configurations the box supports), then one sampled run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pcs
mkdir -p $OUT
METHOD=${PCS_METHOD:-stochastic}
UNIT=${PCS_UNIT:-cycles}
INTERVAL=${PCS_INTERVAL:-1048576}
timeout -k 10 60 rocprofv3 -L > $OUT/list.txt 2>&1
timeout -k 10 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $METHOD --pc-sampling-unit $UNIT \
  --pc-sampling-interval $INTERVAL --output-format csv -d $OUT/run -o pcs -- \
  python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 --pcie-steps 0 > $OUT/bench.json 2> $OUT/bench.err
rc=$?
echo "exit $rc"; tail -5 $OUT/bench.err; ls -laR $OUT/run | head -30
exit $rc
