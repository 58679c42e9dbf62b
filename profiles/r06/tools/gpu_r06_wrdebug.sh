#!/bin/bash
# Round 6 (historical): the wave-private rows variant's parity debug -- world2
# 1080p through the variant builds (wrwait, blk) against the oracle
# (wr_debug.py).  The variant was rejected and its code removed from the
# kernels (archived in ../ab/wave_rows_raster_block.hip.txt), so this script
# only documents what was run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r06/wrdebug
mkdir -p $O
L=$PWD/constructionsceneposeestimation_amd
for v in ${VARIANTS:-base wrwait blk}; do
  if [ $v = base ]; then lib=$L/libcsg.so; else lib=$L/libcsg_$v.so; fi
  CSG_LIB=$lib timeout -k 10 300 python3 -u profiles/r06/tools/wr_debug.py 2>&1 | tee -a $O/wrdebug.txt || exit 1
done
