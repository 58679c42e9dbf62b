#!/bin/bash
# Round 4 (late): PMC passes of the final kernels (pooled work buffers) at the
# bench's launch size, then the N > 1 path at the driver's default sizes on one
# GPU (2 ranks x 2,880 frames per step; 4 ranks x 960), each rank its own shard.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04
mkdir -p $O
ROUND=r04f PASSES="${PASSES:-fetch write valu sq}" bash tools/pmc_profile.sh > $O/pmc_final.log 2>&1 || { tail -20 $O/pmc_final.log; exit 1; }
tail -5 $O/pmc_final.log
port=$((29500 + RANDOM % 1000))
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port bench.py --gpus 2 > $O/rehearsal_2ranks.json 2> $O/rehearsal_2ranks.err || { tail -8 $O/rehearsal_2ranks.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/rehearsal_2ranks.json')); print('N=2', d['value'], d['config']['frames_per_step'], d['verified'], d['shards']['disjoint'])" || exit 1
port=$((29500 + RANDOM % 1000))
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port $port bench.py --gpus 4 --frames-per-step 960 > $O/rehearsal_4ranks.json 2> $O/rehearsal_4ranks.err || { tail -8 $O/rehearsal_4ranks.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/rehearsal_4ranks.json')); print('N=4', d['value'], d['config']['frames_per_step'], d['verified'], d['shards']['disjoint'])"
