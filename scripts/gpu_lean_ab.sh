#!/bin/bash
# Lean-kernel A/B runs (timings only).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "WG_LEAN_PERSIST=0" "WG_LEAN_PERSIST=1" "WG_LEAN=0" "WG_LEAN_PERSIST=0"; do
  echo "$v: $(env $v timeout -k 10 100 python scripts/n_sweep.py 65536 262144 2>/dev/null | tr '\n' ' ')"
done
