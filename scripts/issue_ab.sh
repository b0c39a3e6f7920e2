#!/bin/bash
# Range issue order A/B on one box (profiling aid): bench.py under env variants of the walker-range issue
# (WG_RANGE_ISSUE=seq: range by range; inter: step by step through wg_run_ranges; WG_RANGE_LEAD / WG_RANGE_SKEW_US:
# range 0 ahead by issued steps / by a timed wait), alternating, at the driver's K = 20 and at K = 1,000.
# usage: [BENCH_ARGS="--walkers 4096 --graph"] scripts/issue_ab.sh TAG ROUNDS WORKLOAD NAME:ENV=V,ENV=V ...
set -o pipefail
tag=$1; rounds=$2; wl=$3; shift 3
variants=("$@")
out=gpurun_out/${tag}_issue_ab.jsonl
: > "$out"
for r in $(seq "$rounds"); do
  for k in "20 5" "1000 50"; do
    set -- $k
    for spec in "${variants[@]}"; do
      name=${spec%%:*}; envs=${spec#*:}
      line=$(env ${envs//,/ } timeout -k 10 120 python bench.py --steps "$1" --warmup "$2" --workload "$wl" \
             --no-cpu-baseline --no-control $BENCH_ARGS | tail -1) || exit 1
      echo "{\"round\": $r, \"variant\": \"$name\", \"env\": \"$envs\", \"K\": $1, \"bench\": $line}" >> "$out"
      echo "$r $name K=$1 $(echo "$line" | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')"
    done
  done
done
