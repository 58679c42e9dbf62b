#!/bin/bash
# Round 6: k_setup per-vertex transform (libcsg_sv.so, -DCSG_SETUP_VERTS=1) --
# the parity tests through the variant first, then the A/B against libcsg.so,
# 3 runs each in turn, every line self-verified on 32 frames.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r06/setup_verts
mkdir -p $O
P=$PWD/constructionsceneposeestimation_amd
CSG_LIB=$P/libcsg_sv.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py -x -v --timeout 300 --timeout-method thread > $O/pytest_sv.log 2>&1 || { tail -30 $O/pytest_sv.log; exit 1; }
tail -1 $O/pytest_sv.log
for k in 1 2 3; do
  for v in base sv; do
    lib=$P/libcsg.so; [ $v = sv ] && lib=$P/libcsg_sv.so
    CSG_LIB=$lib timeout -k 10 300 python3 bench.py --pcie-steps 0 --stats-steps 0 > $O/${v}_$k.json 2> $O/${v}_$k.err || { tail -5 $O/${v}_$k.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${v}_$k.json')); print('$v', d['value'], d['stage_ms_per_step'], d['verified']['frames'], d['verified']['bit_exact'])" || exit 1
  done
done
