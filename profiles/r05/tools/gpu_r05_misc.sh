#!/bin/bash
# Round 5: staged-batch size of the 32x16 build (with the label-statistics and
# occlusion legs), and the generator with three renderer contexts.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
REPS=${REPS:-2} STEPS=6 FPS=2880 STATS=2 SKIP_LDS=1 CTR_VARIANTS="" VARIANTS="${VARIANTS:-base ns64 ns56}" bash tools/gpu_variant_ab.sh || exit 1
O=gpurun_out/r05/gen
mkdir -p $O
for R in 3; do
timeout -k 10 300 python3 -u tools/gen_steady.py --frames 20000 --outputs rgb,mask,depth_csv,depth_png --sink discard --renderers $R > $O/steady_no_pointcloud_r$R.json 2> $O/steady_no_pointcloud_r$R.err || { tail -20 $O/steady_no_pointcloud_r$R.err; exit 1; }
cat $O/steady_no_pointcloud_r$R.json
timeout -k 10 400 python3 -u tools/gen_steady.py --frames 20000 --outputs reference --sink discard --renderers $R > $O/steady_reference_r$R.json 2> $O/steady_reference_r$R.err || { tail -20 $O/steady_reference_r$R.err; exit 1; }
cat $O/steady_reference_r$R.json
done
