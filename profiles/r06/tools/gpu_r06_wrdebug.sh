#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r06/wrdebug
mkdir -p $O
L=$PWD/constructionsceneposeestimation_amd
for v in ${VARIANTS:-base wrwait blk}; do
  if [ $v = base ]; then lib=$L/libcsg.so; else lib=$L/libcsg_$v.so; fi
  CSG_LIB=$lib timeout -k 10 300 python3 -u profiles/r06/tools/wr_debug.py 2>&1 | tee -a $O/wrdebug.txt || exit 1
done
