#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r06/wrdebug
mkdir -p $O
L=$PWD/constructionsceneposeestimation_amd
CSG_DEBUG=512 CSG_LIB=$L/libcsg_wrdbg.so REPS=1 timeout -k 10 300 python3 -u profiles/r06/tools/wr_debug.py 2>&1 | tee $O/wrdbg.txt
