#!/bin/bash
# VALU instruction counts and lane utilisation per k_raster ablation setting
# (libcsg_abl.so, CSG_DEBUG bits; one rocprofv3 --pmc pass per setting).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export CSG_LIB=$PWD/constructionsceneposeestimation_amd/libcsg_abl.so
OUT=gpurun_out/abl_valu
mkdir -p $OUT
rc=0
for d in ${DBGS:-0 1 2 4 8 16 256 4096 8192}; do
  CSG_DEBUG=$d timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d $OUT/d$d/pass -o pmc -- python3 bench.py --steps 3 --warmup 1 --frames-per-step ${FPS:-960} --verify-frames 0 --pcie-steps 0 --stats-steps 0 > $OUT/d$d.json 2> $OUT/d$d.err || { rc=$?; break; }
  python3 tools/pmc_summarize.py $OUT/d$d > $OUT/d$d.summary.json && python3 -c "
import json; o=json.load(open('$OUT/d$d.summary.json'))['k_raster']
print('CSG_DEBUG=$d', 'valu=%.3fG' % (o['SQ_INSTS_VALU']/1e9), 'lane_ops=%.1fG' % (o['SQ_THREAD_CYCLES_VALU']/1e9), 'lds=%.3fG' % (o['SQ_INSTS_LDS']/1e9), 'salu=%.3fG' % (o['SQ_INSTS_SALU']/1e9), 'busy=%.3f' % o['valu_busy'], 'util=%.3f' % o['valu_lane_util'])" | tee -a $OUT/valu_per_ablation.txt
done
exit $rc
