#!/bin/bash
# A/B of library variants on bench.py (round 5's tile-shape driver, now the
# generic one): VARIANTS="base name[:ENV=val]..." runs libcsg.so ("base") and
# libcsg_<name>.so (built on the CPU beforehand by tools/build_variant.sh) REPS
# times in turn, each line self-verified on 8 frames; optionally the profiling
# counters per variant (CTR_VARIANTS, CSG_DEBUG=512 builds) and the LDS
# counters per ablation setting (libcsg_abl.so; SKIP_LDS=1 skips them).
# Results: $OUT/tile_ab.txt (default gpurun_out/r05/ab, where round 5's
# scripts under profiles/r05/tools expect them).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r05/ab}
mkdir -p $O
L=$PWD/constructionsceneposeestimation_amd
ARGS="--steps ${STEPS:-8} --warmup 1 --frames-per-step ${FPS:-960} --pcie-steps 0 --stats-steps ${STATS:-0} --cpu-single-frames 1 ${EXTRA}"
# 1. the counters this GPU's profiler offers
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || echo "list-avail failed"
want="SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_ANY SQ_WAVE_CYCLES"
ctrs=""
for c in $want; do grep -q "\b$c\b" $O/avail.txt && ctrs="$ctrs $c"; done
echo "LDS pass counters:$ctrs GRBM_GUI_ACTIVE"
# 2. tile shapes: frames/s, stage times, bin entries (bench line), bit-exact check of 8 frames
if [ "${SKIP_AB:-0}" != 1 ]; then
for rep in $(seq ${REPS:-2}); do
for spec in ${VARIANTS:-base s108 w64h16 w32h16 w16h16}; do
  # name[:VAR=value[:VAR=value]]: library libcsg_<name>.so (base: libcsg.so) with those environment settings
  v=${spec%%:*}; envs=""; [ "$spec" != "$v" ] && envs=$(echo ${spec#*:} | tr ':' ' ')
  tag=$(echo $spec | tr ':=' '__')
  if [ $v = base ]; then lib=$L/libcsg.so; else lib=$L/libcsg_$v.so; fi
  env CSG_LIB=$lib $envs timeout -k 10 300 python3 bench.py $ARGS --verify-frames 8 > $O/tile_$tag.json 2> $O/tile_$tag.err || { echo "$spec FAILED"; tail -5 $O/tile_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/tile_$tag.json')); ws=d.get('with_label_stats') or {}; print('$spec rep $rep', d['value'], d['stage_ms_per_step'], 'recs/frame', d['records_per_frame'], 'bins/frame', d['bin_entries_per_frame'], 'exact', d['verified']['bit_exact'], d['verified']['frames'], 'stats', ws.get('value'), 'occl', (ws.get('with_occlusion_and_depth_png') or {}).get('value'))" | tee -a $O/tile_ab.txt
done
done
fi
# 3. level-2 lanes and staged records per shape (profiling counters, CSG_DEBUG 512)
for v in ${CTR_VARIANTS-abl abl_w64h16 abl_w32h16 abl_w16h16}; do
  CSG_LIB=$L/libcsg_$v.so CSG_DEBUG=512 timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --frames-per-step 240 --verify-frames 0 --pcie-steps 0 --stats-steps 0 --size-work 0 > $O/ctr_$v.json 2> $O/ctr_$v.err || { echo "$v counters FAILED"; tail -5 $O/ctr_$v.err; exit 1; }
  echo "$v $(grep '\[csg\] staged_recs' $O/ctr_$v.err | tail -1)" | tee -a $O/tile_counters.txt
done
# 4. LDS counters per ablation setting (production-equivalent kernels with CSG_ABLATION=1)
if [ -n "$ctrs" ] && [ "${SKIP_LDS:-0}" != 1 ]; then
for d in ${DBGS:-0 1 4 8 256 8192}; do
  CSG_LIB=$L/libcsg_abl.so CSG_DEBUG=$d timeout -s KILL 180 rocprofv3 --pmc $ctrs GRBM_GUI_ACTIVE --output-format csv -d $O/lds${LDS_TAG}_d$d/pass -o pmc -- python3 bench.py --steps 3 --warmup 1 --frames-per-step 960 --verify-frames 0 --pcie-steps 0 --stats-steps 0 > $O/lds${LDS_TAG}_d$d.json 2> $O/lds${LDS_TAG}_d$d.err || { echo "LDS pass $d FAILED"; tail -5 $O/lds${LDS_TAG}_d$d.err; exit 1; }
  python3 tools/pmc_summarize.py $O/lds${LDS_TAG}_d$d > $O/lds${LDS_TAG}_d$d.summary.json && python3 -c "
import json; o=json.load(open('$O/lds${LDS_TAG}_d$d.summary.json'))['k_raster']
print('${LDS_TAG} CSG_DEBUG=$d', {k: round(v/1e6, 2) for k, v in o.items() if k.startswith('SQ_') and not k.endswith('_n')})" | tee -a $O/lds_counters.txt
done
fi
