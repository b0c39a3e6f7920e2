#!/bin/bash
# Lean-kernel A/B: waves per workgroup, then PMC passes of the default kernel.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in 1 2 4; do echo "waves/wg $w: $(WG_LEAN_WAVES=$w timeout -k 10 100 python scripts/sweep_w.py one 2>/dev/null)"; done
bash scripts/gpu_pmc.sh lean
