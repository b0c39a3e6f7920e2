S=scripts/gpu_session.sh
$S "r05z_graph_tests:400:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_policy_loop.py tests/test_gpu_prepared.py tests/test_gpu_ragged.py -q -x --timeout 120 --timeout-method thread -k 'graph or policy or prepared or lanes or rollout'" \
   "r05z_bench_graph:300:python bench.py --graph --steps 200 --warmup 20 --no-cpu-baseline --no-control" \
   "r05z_bench_graph_ragged:300:python bench.py --workload ragged --graph --steps 200 --warmup 20 --no-cpu-baseline --no-control" \
   "r05z_bench_graph_k20:300:python bench.py --graph --steps 20 --warmup 5 --no-cpu-baseline --no-control" \
   "r05z_bench_k20:300:python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-control" \
   "r05z_bench_balance:300:python bench.py --workload balance --walkers 4096 --graph --resident --steps 1000 --warmup 100 --no-cpu-baseline"
