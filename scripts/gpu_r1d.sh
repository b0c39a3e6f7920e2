#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout_s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -n 12 "gpurun_out/$name.log"
  if [ $rc -ge 2 ] && [ $rc -ne 5 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step variants 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 400 --timeout-method thread -k "variants or golden"
step rev_ab 300 python -u scripts/rev_ab.py 3 build_ablate/lib_rev_3655086.so build_ablate/lib_rev_head.so
step lean_ab 300 python -u scripts/lean_ab.py 3 lean pf quo quo_pf lean_w1
