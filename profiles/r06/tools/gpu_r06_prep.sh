#!/bin/bash
# Round 6: generate() with batch preparation in worker processes (prep_pool.py):
# the GPU test that the files are identical, then the steady-state no-point-cloud
# run with 2 prep workers and with none, in turn, on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r06/prep
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_prep_workers.py -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
NO_PC=rgb,mask,depth_csv,depth_png
for k in 1 2; do
  for p in 2 0; do
    timeout -k 10 300 python3 -u tools/gen_steady.py --frames ${FRAMES:-20000} --outputs $NO_PC --sink discard --prep-workers $p > $O/steady_p${p}_$k.json 2> $O/steady_p${p}_$k.err || { tail -20 $O/steady_p${p}_$k.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/steady_p${p}_$k.json')); print('prep', $p, d['frames_per_s'], d['writer_busy'], d['render_busy'], d['render_thread'], d['d2h_gbs'])"
  done
done
