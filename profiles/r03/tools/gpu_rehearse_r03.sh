#!/bin/bash
# Multi-rank rehearsal of the driver's N>1 bench launch on a 1-GPU box (ranks share the device;
# frames per step scaled down so the ranks' work buffers fit in one GPU's memory).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rc=0
for n in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 10 --warmup 2 --frames-per-step $((960 * 2 / n)) > gpurun_out/rehearse_$n.json 2> gpurun_out/rehearse_$n.err || { rc=$?; break; }
done
for n in 2 4; do python3 -c "import json; d=json.load(open('gpurun_out/rehearse_$n.json')); print($n, d['value'], d['n_gpus'], d.get('verified'))" 2>/dev/null; done
exit $rc
