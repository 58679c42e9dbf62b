#!/bin/bash
# Round 6 k_raster A/B: base (this tree), pf (CSG_PREFETCH_BIN=1: record ids one
# batch ahead), wr (CSG_WAVE_ROWS=1: wave-private rows; not bit-exact yet, so
# its lines run without the oracle check and say so), in turn, REPS times, at
# the bench's 2,880 frames per step; then the GPU tests touched this round.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r06/b2
mkdir -p $O
L=$PWD/constructionsceneposeestimation_amd
ARGS="--steps 6 --warmup 1 --frames-per-step 2880 --pcie-steps 0 --stats-steps 0 --cpu-single-frames 1"
for rep in $(seq ${REPS:-3}); do
  for v in ${VARIANTS:-base pf wr}; do
    if [ $v = base ]; then lib=$L/libcsg.so; else lib=$L/libcsg_$v.so; fi
    vf=8; [ $v = wr ] && vf=0
    CSG_LIB=$lib timeout -k 10 300 python3 bench.py $ARGS --verify-frames $vf > $O/ab_$v.json 2> $O/ab_$v.err || { echo "$v FAILED"; tail -5 $O/ab_$v.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/ab_$v.json')); print('$v rep $rep', d['value'], d['stage_ms_per_step'], 'verified', d['verified']['frames'])" | tee -a $O/ab.txt
  done
done
if [ "${TESTS:-1}" = 1 ]; then
timeout -k 10 1200 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_id_wire.py tests/test_gpu_retry.py tests/test_gpu_max_frame.py tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_async.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
fi
