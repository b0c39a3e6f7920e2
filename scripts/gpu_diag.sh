#!/bin/bash
# Diagnostic session: phase ablation, W sweep, memory skeleton.  Each step under its own limit.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
echo "== membench"; timeout -k 10 120 ./build_ablate/membench 2>&1 | tee gpurun_out/membench.log || exit 1
echo "== ablate";   timeout -k 10 400 python scripts/ablate.py run 2>&1 | tee gpurun_out/ablate.log || exit 1
echo "== W sweep";  timeout -k 10 400 python scripts/sweep_w.py 8 12 16 24 32 2>&1 | tee gpurun_out/sweep.log || exit 1
