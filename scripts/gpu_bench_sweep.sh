#!/bin/bash
# bench.py timing vs steps / warmup on one box (why the in-process A/B and bench.py differ)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for sw in "100 30" "300 30" "1000 30" "300 300" "300 1000"; do
  set -- $sw
  timeout -k 10 120 python bench.py --steps $1 --warmup $2 --no-cpu-baseline --no-control > gpurun_out/bs_$1_$2.log 2>&1 || exit 1
  echo "steps $1 warmup $2: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bs_$1_$2.log)"
done
timeout -k 10 120 python scripts/lean_ab.py 3 lean > gpurun_out/bs_ab.log 2>&1 && grep median gpurun_out/bs_ab.log
