#!/bin/bash
# Final session of the round: parity suite, smoke, bench (CPU baseline), rocprof kernel stats, PMC passes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout_s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -n 4 "gpurun_out/$name.log"
  if [ $rc -ge 2 ] && [ $rc -ne 5 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 400 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 500 --warmup 50
step bench_balance 300 python bench.py --steps 500 --warmup 50 --workload balance --walkers 65536 --no-cpu-baseline
step bench_ragged 300 python bench.py --steps 300 --warmup 30 --workload ragged --walkers 65536 --no-cpu-baseline
step rocprof_trace 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline
step pmc 900 bash scripts/gpu_pmc.sh pmc
