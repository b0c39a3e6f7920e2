#!/bin/bash
# plain bench.py against `torchrun --nproc-per-node 1 bench.py --gpus 1` (the driver's world-1 command), interleaved
# on one box, K / W from KS (default "20 5"), ROUNDS rounds: gpurun_out/<tag>_torchrun_ab.jsonl (profiling aid).
# Variants NAME:plain|torchrun[:ENV=V,ENV=V] (default "plain:plain torchrun:torchrun").
# usage: [KS="20 5"] scripts/torchrun_ab.sh TAG ROUNDS [VARIANT ...]
set -o pipefail
tag=$1; rounds=$2; shift 2
variants=("$@")
[ ${#variants[@]} -eq 0 ] && variants=("plain:plain" "torchrun:torchrun")
out=gpurun_out/${tag}_torchrun_ab.jsonl
: > "$out"
read -r K W <<< "${KS:-20 5}"
for r in $(seq "$rounds"); do
  for spec in "${variants[@]}"; do
    IFS=: read -r name mode envs <<< "$spec"
    if [ "$mode" = plain ]; then
      line=$(env ${envs//,/ } timeout -k 10 120 python bench.py --steps $K --warmup $W --no-cpu-baseline --no-control \
             | tail -1) || exit 1
    else
      line=$(env ${envs//,/ } timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
             --master-addr 127.0.0.1 --master-port $((29700 + r)) bench.py --gpus 1 --steps $K --warmup $W \
             --no-cpu-baseline --no-control 2>/dev/null | grep '^{' | tail -1) || exit 1
    fi
    echo "{\"round\": $r, \"variant\": \"$name\", \"env\": \"$envs\", \"K\": $K, \"bench\": $line}" >> "$out"
    echo "$r $name $(echo "$line" | python -c 'import json,sys; d=json.load(sys.stdin); t=d["timing"]; print(d["ms_per_step"], t["kernel_ms_per_step_events"], t.get("comm_live_ms_per_step"))')"
  done
done
