#!/bin/bash
# k_raster<true> kernel time per library variant (rocprofv3 kernel stats):
#   LIBS="cov covnm" bash tools/prof_cov.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ${LIBS}; do
  CSG_LIB=$PWD/constructionsceneposeestimation_amd/libcsg_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pc_$v -o run -- python3 bench.py --verify-frames 0 --pcie-steps 0 --stats-steps ${STATS:-6} --steps 5 > gpurun_out/pc_$v.json 2>gpurun_out/pc_$v.err || { echo "$v FAILED"; tail -5 gpurun_out/pc_$v.err; exit 1; }
  f=$(find gpurun_out/pc_$v -name '*kernel_stats.csv' | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'raster' in r['Name'] or 'depth' in r['Name']: print('$v', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e6, 3))"
done
