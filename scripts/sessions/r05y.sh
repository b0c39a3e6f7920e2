S=scripts/gpu_session.sh
$S "r05y_bench_graph:300:python bench.py --graph --steps 200 --warmup 20 --no-cpu-baseline --no-control" \
   "r05y_bench_graph_ragged:300:python bench.py --workload ragged --graph --steps 200 --warmup 20 --no-cpu-baseline --no-control"
