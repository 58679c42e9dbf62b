#!/bin/bash
# A/B of k_raster variants: parity (GPU tests) and bench, one GPU session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VARS=${VARS:-"0 1 2"}
for v in $VARS; do
  CSG_VARIANT=$v timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x > gpurun_out/ab_test_$v.log 2>&1 || { echo "variant $v FAILED parity"; tail -20 gpurun_out/ab_test_$v.log; exit 1; }
done
for rep in 1 2; do
for v in $VARS; do
  CSG_VARIANT=$v timeout -k 10 200 python bench.py --cpu-sample 0 --steps 20 > gpurun_out/ab_$v.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); print('variant $v', d['value'], d['stage_ms_per_step'])"
done
done
