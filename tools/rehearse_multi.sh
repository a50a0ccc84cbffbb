#!/bin/bash
# Rehearsal of bench.py's N>1 path on a 1-GPU box: 2 ranks share cuda:0 over gloo (RCCL refuses two ranks on one
# device).  Exercises sharding, the aggregation / dense-plane / sparse-group merges and max-over-ranks timing.
set -euo pipefail
mkdir -p gpurun_out/multi
export PGX_DIST_BACKEND=gloo
for wl in "c2 --rows 20000000" "c5 --rows 200000" "c3 --rows 2000000" "c3m2 --rows 1000000" "c3f --rows 1000000"; do
  name=${wl%% *}
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --workload $wl \
    > gpurun_out/multi/$name.log 2>&1
done
