#!/bin/bash
# One GPU session made of named steps (replaces round 5's 35 one-off scripts/sessions/r05*.sh):
#     TAG=r06a bash scripts/session.sh gputest smoke bench_k20 nccl1 ...
# Each step runs under scripts/gpu_session.sh (its own time limit; a crash, abort or timeout ends the session) and
# writes gpurun_out/${TAG}_<step>.log (rocprofv3 steps: gpurun_out/${TAG}_<step>/); scripts/keep_profiles.py ${TAG}_
# then copies the judged pieces into profiles/.  A step that is not a preset name is taken as "name:timeout:command".
cd "${GRAFT_REPO_ROOT:-/root/repo}"
t=${TAG:?set TAG, e.g. TAG=r06a}
W1PORT=${W1PORT:-29631}
steps=()
for s in "$@"; do
  case "$s" in
    gputest)         steps+=("${t}_gputest:420:python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread");;
    smoke)           steps+=("${t}_smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'");;
    bench_k20)       steps+=("${t}_bench_k20:240:python bench.py --gpus 1 --steps 20 --warmup 5");;
    bench)           steps+=("${t}_bench:360:python bench.py --resident");;
    nccl1)           steps+=("${t}_nccl1:300:python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port ${W1PORT} bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline");;
    prof_canonical)  steps+=("${t}_prof_canonical:300:rocprofv3 --kernel-trace --stats -d gpurun_out/${t}_prof_canonical -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 200 --sustained-steps 0");;
    bench_ragged)    steps+=("${t}_bench_ragged:400:python bench.py --workload ragged");;
    prof_ragged)     steps+=("${t}_prof_ragged:300:rocprofv3 --kernel-trace --stats -d gpurun_out/${t}_prof_ragged -o run --output-format csv -- python bench.py --workload ragged --no-cpu-baseline --steps 200 --sustained-steps 0");;
    bench_balance)   steps+=("${t}_bench_balance4096:300:python bench.py --workload balance --walkers 4096 --graph --resident --steps 1000 --warmup 100");;
    bench_balance_direct) steps+=("${t}_bench_balance4096_direct:300:python bench.py --workload balance --walkers 4096 --resident --steps 1000 --warmup 100 --no-cpu-baseline");;
    bench_chain)     steps+=("${t}_bench_chain:400:python bench.py --workload chain --walkers 4096 --chain-points 100 --steps 100 --warmup 10 --cpu-seconds 10");;
    bench_perfdemo)  steps+=("${t}_bench_perfdemo:400:python bench.py --workload perfdemo --walkers 4096 --chain-points 100 --steps 100 --warmup 10 --cpu-seconds 10");;
    pmc)             steps+=("${t}_pmc:400:bash scripts/gpu_pmc.sh ${t}_pmc_canonical && WG_WORKLOAD=ragged bash scripts/gpu_pmc.sh ${t}_pmc_ragged");;
    pmc_valu)        steps+=("${t}_pmc_valu:300:bash scripts/gpu_pmc.sh ${t}_valu_canonical valu");;
    *)               steps+=("$s");;
  esac
done
exec bash scripts/gpu_session.sh "${steps[@]}"
