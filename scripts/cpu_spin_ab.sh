#!/bin/bash
# Does host CPU load change the GPU's burst clock?  bench.py at the driver's K = 20, alternating plain runs with runs
# beside N busy-spinning CPU processes (each killed by PID after its run).  usage: cpu_spin_ab.sh TAG ROUNDS NSPIN
tag=$1; rounds=$2; nspin=$3
out=gpurun_out/${tag}_spin_ab.jsonl
: > "$out"
for r in $(seq "$rounds"); do
  for v in plain spin; do
    pids=()
    if [ "$v" = spin ]; then
      for i in $(seq "$nspin"); do python3 -c "while True: pass" & pids+=($!); done
      sleep 1
    fi
    line=$(timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-control | tail -1)
    rc=$?
    for p in "${pids[@]}"; do kill "$p"; done
    wait 2>/dev/null
    [ $rc -eq 0 ] || exit 1
    echo "{\"round\": $r, \"variant\": \"$v\", \"nspin\": $nspin, \"bench\": $line}" >> "$out"
    echo "$r $v $(echo "$line" | python -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"])')"
  done
done
