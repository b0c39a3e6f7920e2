bash scripts/gpu_session.sh \
 "r03zk_gputest_floor:200:python -u -m pytest tests/test_gpu_parity.py -x -q -k 'launch_floor or full_size' --timeout 150 --timeout-method thread" \
 "r03zk_bench_balance4096:200:python bench.py --workload balance --walkers 4096 --graph --steps 1000 --warmup 100 --no-cpu-baseline" \
 "r03zk_bench_balance4096_nograph:200:python bench.py --workload balance --walkers 4096 --steps 1000 --warmup 100 --no-cpu-baseline"
