#!/bin/bash
# GPU session: parity tests, smoke, bench, rocprof kernel trace.  Each GPU step has its own time
# limit; a crash/abort/timeout (rc >= 124) ends the session; plain test failures (rc 1) do not.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout_s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ge 2 ] && [ $rc -ne 5 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 300 --warmup 30
step bench_lanes1 600 env WG_LANES=1 python bench.py --steps 300 --warmup 30 --no-cpu-baseline
step bench_balance 600 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --workload balance
step bench_ragged 600 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --workload ragged
step rocprof_trace 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-control
step trace_span 60 python scripts/trace_span.py gpurun_out/prof/run_kernel_trace.csv 200
step rocprof_trace_l1 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_l1 -o run --output-format csv -- python scripts/prof_run.py
if [ -n "$WG_AB" ]; then  # A/B: barrier kernel vs lean
  step bench_barrier 600 env WG_LEAN=0 python bench.py --steps 300 --warmup 30 --no-cpu-baseline
fi
