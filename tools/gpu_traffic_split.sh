#!/bin/bash
# k_raster's HBM-side traffic split per phase.  The ablation build
# (libcsg_abl.so: `tools/build_variant.sh abl - -DCSG_ABLATION=1`) with the
# CSG_DEBUG bits of DESIGN §5 (0 all, 1 no resolve, 8 no level-2 fragments,
# 256 no level 1, 2 empty-tile resolve only); per setting three rocprofv3
# --pmc passes of their own: FETCH_SIZE, WRITE_SIZE, and the L2 request
# counters (TCC_EA0_RDREQ: all L2 read misses, TCC_EA0_RDREQ_DRAM: those the
# fabric sent to DRAM, i.e. missed in the Infinity Cache too).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export CSG_LIB=$PWD/constructionsceneposeestimation_amd/libcsg_abl.so
OUT=${OUT:-gpurun_out/traffic}
mkdir -p $OUT
ARGS="--steps 3 --warmup 1 --frames-per-step ${FPS:-960} --verify-frames 0 --pcie-steps 0 --stats-steps 0"
rc=0
for d in ${DBGS:-0 1 8 256 2}; do
  for p in fetch write tcc; do
    case $p in
      fetch) C="FETCH_SIZE" ;;
      write) C="WRITE_SIZE" ;;
      tcc) C="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum" ;;
    esac
    CSG_DEBUG=$d timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/d$d/$p -o pmc -- python3 bench.py $ARGS > $OUT/d$d.$p.json 2> $OUT/d$d.$p.err || { rc=$?; echo "d$d $p failed rc=$rc"; tail -5 $OUT/d$d.$p.err; exit $rc; }
  done
  python3 tools/pmc_summarize.py $OUT/d$d > $OUT/d$d.summary.json || exit 1
  python3 -c "
import json; o=json.load(open('$OUT/d$d.summary.json'))['k_raster']
print('CSG_DEBUG=$d', json.dumps({k: o.get(k) for k in ('FETCH_SIZE','WRITE_SIZE','TCC_EA0_RDREQ_sum','TCC_EA0_RDREQ_DRAM_sum','TCC_HIT_sum','TCC_MISS_sum','hbm_bytes_per_launch')}))" | tee -a $OUT/traffic_per_ablation.txt
done
exit $rc
