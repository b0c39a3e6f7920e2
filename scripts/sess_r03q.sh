bash scripts/gpu_session.sh \
 "r03q_gputest:500:python -u -m pytest tests -m gpu -q --timeout 250 --timeout-method thread" \
 "r03q_smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "r03q_bench_ragged:300:python bench.py --workload ragged --no-cpu-baseline" \
 "r03q_bench_balance65536:200:python bench.py --workload balance --no-cpu-baseline" \
 "r03q_bench_chain:400:python bench.py --workload chain --walkers 4096 --chain-points 100 --steps 100 --warmup 10 --cpu-seconds 10" \
 "r03q_bench_perfdemo:400:python bench.py --workload perfdemo --walkers 4096 --chain-points 100 --steps 100 --warmup 10 --no-cpu-baseline" \
 "r03q_bench_nccl1:300:python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --no-cpu-baseline" \
 "r03q_pmc_ragged:200:WG_WORKLOAD=ragged bash scripts/gpu_pmc.sh r03q_pmc_ragged"
