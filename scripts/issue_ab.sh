#!/bin/bash
# Range issue order A/B on one box (profiling aid): bench.py with the walker ranges issued step by step
# (wg_run_ranges, the default) against range by range (WG_RANGE_ISSUE=seq), alternating, at the driver's K = 20
# and at K = 1,000.  usage: scripts/issue_ab.sh TAG [rounds] [workload]
set -o pipefail
tag=$1; rounds=${2:-3}; wl=${3:-canonical}
out=gpurun_out/${tag}_issue_ab.jsonl
: > "$out"
for r in $(seq "$rounds"); do
  for k in "20 5" "1000 50"; do
    set -- $k
    for v in inter seq; do
      line=$(WG_RANGE_ISSUE=$v timeout -k 10 120 python bench.py --steps "$1" --warmup "$2" --workload "$wl" \
             --no-cpu-baseline --no-control | tail -1) || exit 1
      echo "{\"round\": $r, \"issue\": \"$v\", \"K\": $1, \"bench\": $line}" >> "$out"
      echo "$r $v K=$1 $(echo "$line" | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')"
    done
  done
done
