#!/bin/bash
# SQ counter calibration (tools/calib_valu.hip) and k_raster's wave-cycle split
# per ablation phase (libcsg_abl.so: CSG_ABLATION=1, built on the CPU with
#   tools/build_variant.sh abl - -DCSG_ABLATION=1).
# One counter group per rocprofv3 run, no trace domains beside --pmc.
# Output: $OUT (default gpurun_out/r06/calib); summary: tools/calib_valu_summary.py $OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r06/calib}
mkdir -p $O
L=$PWD/constructionsceneposeestimation_amd
[ -x tools/calib_valu ] || { echo "tools/calib_valu missing (build it on the CPU)"; exit 1; }
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || echo "list-avail failed"
grep -o 'Counter_Name *: *[A-Za-z0-9_]*' $O/avail.txt | awk '{print $3}' | sort -u > $O/counter_names.txt
grep -iE 'BARRIER|WAIT|SLEEP|IFETCH' $O/counter_names.txt > $O/wait_counters.txt || true
echo "wait-like counters: $(tr '\n' ' ' < $O/wait_counters.txt)"
PA="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
PB="SQ_WAVES SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
# pass C: SQ counters that name barriers / sleeps, if this profiler offers any (at most 6)
PC=""
for c in $(grep -iE '^SQ_.*(BARRIER|SLEEP)' $O/counter_names.txt | head -6); do PC="$PC $c"; done
[ -n "$PC" ] && PC="SQ_WAVE_CYCLES$PC GRBM_GUI_ACTIVE"
echo "pass C:$PC"
# 1. the calibration kernels: one timing run, then the counter passes
timeout -k 10 120 ./tools/calib_valu > $O/calib.json || { echo "calib_valu failed"; exit 1; }
cat $O/calib.json
for p in A B C; do
  eval ctrs=\$P$p
  [ -z "$ctrs" ] && continue
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d $O/calib_$p -o pmc -- ./tools/calib_valu > $O/calib_$p.json 2> $O/calib_$p.err || { echo "calib pass $p failed"; tail -5 $O/calib_$p.err; exit 1; }
done
# 2. k_raster per ablation phase (CSG_DEBUG bits, tools/ablate.sh): 0 all, 1 no resolve,
#    8 no level-2 items, 256 no level 1 (staging only), 2 empty tiles (fixed cost + background)
[ -f $L/libcsg_abl.so ] || { echo "libcsg_abl.so missing"; exit 1; }
ARGS="--steps 2 --warmup 1 --frames-per-step ${FPS:-960} --verify-frames 0 --pcie-steps 0 --stats-steps 0"
for d in ${DBGS:-0 1 8 256 2}; do
  for p in A ${RASTER_PASSES:-C}; do
    eval ctrs=\$P$p
    [ -z "$ctrs" ] && continue
    CSG_LIB=$L/libcsg_abl.so CSG_DEBUG=$d timeout -s KILL 240 rocprofv3 --pmc $ctrs --output-format csv -d $O/raster_d${d}_$p -o pmc -- python3 bench.py $ARGS > $O/raster_d${d}_$p.json 2> $O/raster_d${d}_$p.err || { echo "raster pass d=$d $p failed"; tail -5 $O/raster_d${d}_$p.err; exit 1; }
    echo "raster d=$d pass $p done"
  done
done
# 3. the production library's k_raster / k_setup at the bench's launch size (pass A and B)
for p in A B; do
  eval ctrs=\$P$p
  timeout -s KILL 300 rocprofv3 --pmc $ctrs --output-format csv -d $O/prod_$p -o pmc -- python3 bench.py --steps 2 --warmup 1 --verify-frames 0 --pcie-steps 0 --stats-steps 0 > $O/prod_$p.json 2> $O/prod_$p.err || { echo "prod pass $p failed"; tail -5 $O/prod_$p.err; exit 1; }
done
python3 tools/calib_valu_summary.py $O > $O/summary.json && cat $O/summary.json
