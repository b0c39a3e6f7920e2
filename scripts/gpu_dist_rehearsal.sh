#!/bin/bash
# Rehearse bench.py's multi-rank path (barrier, max-over-ranks time, rollout-end gather, rank-0 JSON) with 2
# ranks sharing the one GPU of a gpurun box over gloo; the driver's N-GPU runs use RCCL (nccl) instead.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
WG_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 100 --warmup 10 > gpurun_out/dist2g.log 2>&1
