#!/bin/bash
# Bench lines for every workload + rocprofv3 kernel-trace summaries of the single-launch (--lanes 1) runs.
# usage: gpu_bench_all.sh <tag>   (outputs under gpurun_out/<tag>_*)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
t=${1:-r02}
S=scripts/gpu_session.sh
$S "${t}_bench_canonical:300:python bench.py --resident" \
   "${t}_prof_canonical:300:rocprofv3 --kernel-trace --stats -d gpurun_out/${t}_prof_canonical -o run --output-format csv -- python bench.py --no-cpu-baseline" \
   "${t}_bench_ragged:400:python bench.py --workload ragged" \
   "${t}_prof_ragged:300:rocprofv3 --kernel-trace --stats -d gpurun_out/${t}_prof_ragged -o run --output-format csv -- python bench.py --workload ragged --no-cpu-baseline" \
   "${t}_bench_balance4096:300:python bench.py --workload balance --walkers 4096 --graph --steps 1000 --warmup 100" \
   "${t}_bench_balance65536:300:python bench.py --workload balance --no-cpu-baseline" \
   "${t}_bench_chain:400:python bench.py --workload chain --walkers 4096 --chain-points 100 --steps 100 --warmup 10 --cpu-seconds 10"
