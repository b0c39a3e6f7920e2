#!/bin/bash
# Check of the LDS-address-space carve fix: parity suite, canonical and ragged bench lines.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout_s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -n 3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
step bench 300 python bench.py --steps 500 --warmup 50 --no-cpu-baseline
step bench_ragged 300 python bench.py --steps 300 --warmup 30 --workload ragged --walkers 65536 --no-cpu-baseline
step bench_persist 300 env WG_LEAN_PERSIST=1 python bench.py --steps 300 --warmup 30 --no-cpu-baseline
