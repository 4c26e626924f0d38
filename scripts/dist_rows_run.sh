#!/bin/bash
# Row-shard whole layers: 2-rank gloo rehearsals on one GPU (parity vs 1 device), then per-rank
# compute probes of an 8-way cut (rank 0's shard alone) for both layouts, and the 1-GPU forward.
set -o pipefail
mkdir -p gpurun_out
run2() {
  GTA_DIST_BACKEND=gloo GTA_SINGLE_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 scripts/dist_layers.py "$@"
}
run2 gcn-cora gat8-flickr sage-reddit gat8-reddit gin-products --reps 2 --layout rows > gpurun_out/dl_rows2.log 2>&1 || exit $?
run2 gcn-cora gin-products --reps 2 --layout rows --no-replicate > gpurun_out/dl_rows2_allgather.log 2>&1 || exit $?
for L in rows cols; do
  timeout -k 10 300 python scripts/dist_layers.py sage-reddit gat8-reddit gin-products --reps 5 --layout $L --probe 8 \
    > gpurun_out/dl_${L}_probe8.log 2>&1 || exit $?
done
timeout -k 10 300 python scripts/dist_layers.py sage-reddit gat8-reddit gin-products --reps 5 --layout rows \
  > gpurun_out/dl_rows1.log 2>&1
