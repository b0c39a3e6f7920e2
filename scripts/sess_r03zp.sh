bash scripts/gpu_session.sh \
 "r03zp_gputest:500:python -u -m pytest tests -m gpu -q --timeout 250 --timeout-method thread" \
 "r03zp_smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "r03zp_bench:300:python bench.py --resident" \
 "r03zp_bench_k20:300:python bench.py --steps 20 --warmup 5 --no-cpu-baseline" \
 "r03zp_prof_canonical:300:rocprofv3 --kernel-trace --stats -d gpurun_out/r03zp_prof_canonical -o run --output-format csv -- python bench.py --no-cpu-baseline" \
 "r03zp_bench_ragged:300:python bench.py --workload ragged --no-cpu-baseline" \
 "r03zp_bench_balance4096:200:python bench.py --workload balance --walkers 4096 --graph --steps 1000 --warmup 100 --no-cpu-baseline" \
 "r03zp_bench_nccl1:300:python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --no-cpu-baseline"
