#!/bin/bash
# bench.py under env variants, alternating, on one box (profiling aid): round 4's range issue order A/B
# (WG_RANGE_ISSUE=seq: range by range; inter: step by step through wg_run_ranges) and round 5's world-1 / device warm-up
# A/B (WORLD_SIZE=1,RANK=0,LOCAL_RANK=0,MASTER_ADDR=127.0.0.1,MASTER_PORT=P: bench.py's torch.distributed path without
# the launcher; WG_BENCH_WARM_MS).  K / W pairs from KS (default "20 5;1000 50").
# usage: [KS="20 5"] [BENCH_ARGS="--walkers 4096 --graph"] scripts/issue_ab.sh TAG ROUNDS WORKLOAD NAME:ENV=V,ENV=V ...
set -o pipefail
tag=$1; rounds=$2; wl=$3; shift 3
variants=("$@")
out=gpurun_out/${tag}_issue_ab.jsonl
: > "$out"
IFS=';' read -ra kws <<< "${KS:-20 5;1000 50}"
for r in $(seq "$rounds"); do
  for k in "${kws[@]}"; do
    set -- $k
    for spec in "${variants[@]}"; do
      name=${spec%%:*}; envs=${spec#*:}
      line=$(env ${envs//,/ } timeout -k 10 120 python bench.py --steps "$1" --warmup "$2" --workload "$wl" \
             --no-cpu-baseline --no-control $BENCH_ARGS | tail -1) || exit 1
      echo "{\"round\": $r, \"variant\": \"$name\", \"env\": \"$envs\", \"K\": $1, \"bench\": $line}" >> "$out"
      echo "$r $name K=$1 $(echo "$line" | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d.get("timing", {}).get("kernel_ms_per_step_events"))')"
    done
  done
done
