bash scripts/gpu_session.sh \
 "r03w_gputest:500:python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread" \
 "r03w_bench_chain:400:python bench.py --workload chain --walkers 4096 --chain-points 100 --steps 100 --warmup 10 --cpu-seconds 10" \
 "r03w_bench_perfdemo:400:python bench.py --workload perfdemo --walkers 4096 --chain-points 100 --steps 100 --warmup 10 --no-cpu-baseline"
