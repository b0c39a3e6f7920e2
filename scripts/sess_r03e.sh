bash scripts/gpu_session.sh \
 "r03e_gputest:600:python -u -m pytest tests -m gpu -q --timeout 250 --timeout-method thread" \
 "r03e_ab_canon:300:python scripts/variant_ab.py run 5 canonical base: xl:WG_XCD=3" \
 "r03e_ab_ragged:300:python scripts/variant_ab.py run 5 ragged base:" \
 "r03e_ab_bal4096:200:WG_N=4096 python scripts/variant_ab.py run 5 balance base: xl:WG_XCD=3" \
 "r03e_bench:240:python bench.py --no-cpu-baseline" \
 "r03e_bench_perfdemo:240:python bench.py --workload perfdemo --walkers 4096 --chain-points 100 --steps 100 --warmup 10 --no-cpu-baseline"
