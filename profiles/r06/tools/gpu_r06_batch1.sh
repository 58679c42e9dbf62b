#!/bin/bash
# Round 6, first full check: the wave-rows debug build's coverage report, the
# GPU tests touched this round, then the staging-prefetch A/B (old = round-5
# kernels, base = this tree, pf = CSG_PREFETCH_BIN=1), each line verified.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r06/b1
mkdir -p $O
L=$PWD/constructionsceneposeestimation_amd
CSG_DEBUG=512 CSG_LIB=$L/libcsg_wrdbg.so REPS=1 timeout -k 10 300 python3 -u profiles/r06/tools/wr_debug.py > $O/wrdbg.txt 2>&1
echo "wrdbg rc=$?"; grep -E "staged_recs|total" $O/wrdbg.txt | head -5 | cut -c1-400
OUT=$O VARIANTS="${VARIANTS:-old base pf}" REPS=${REPS:-3} FPS=2880 STEPS=6 SKIP_LDS=1 CTR_VARIANTS="" bash tools/gpu_variant_ab.sh || exit 1
timeout -k 10 1200 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_id_wire.py tests/test_gpu_retry.py tests/test_gpu_max_frame.py tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_async.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
