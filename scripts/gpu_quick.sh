#!/bin/bash
# Quick GPU loop: parity tests, bench A/B, stamps.  Stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; tail -n ${TAILN:-4} "gpurun_out/$name.log"; echo "   rc=$rc"; if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi; return 0; }
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run bench_lean 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline
WG_LEAN=0 run bench_old 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline
TAILN=20 run stamps 120 python scripts/stamps.py run
