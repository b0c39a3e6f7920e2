bash scripts/gpu_session.sh \
 "r03zg_gputest:500:python -u -m pytest tests -m gpu -q --timeout 250 --timeout-method thread" \
 "r03zg_smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "r03zg_bench:300:python bench.py --resident" \
 "r03zg_prof_canonical:300:rocprofv3 --kernel-trace --stats -d gpurun_out/r03zg_prof_canonical -o run --output-format csv -- python bench.py --no-cpu-baseline" \
 "r03zg_bench_ragged:300:python bench.py --workload ragged --no-cpu-baseline" \
 "r03zg_prof_ragged:300:rocprofv3 --kernel-trace --stats -d gpurun_out/r03zg_prof_ragged -o run --output-format csv -- python bench.py --workload ragged --no-cpu-baseline" \
 "r03zg_bench_balance4096:200:python bench.py --workload balance --walkers 4096 --graph --steps 1000 --warmup 100 --no-cpu-baseline" \
 "r03zg_bench_chain:400:python bench.py --workload chain --walkers 4096 --chain-points 100 --steps 100 --warmup 10 --cpu-seconds 10" \
 "r03zg_bench_perfdemo:400:python bench.py --workload perfdemo --walkers 4096 --chain-points 100 --steps 100 --warmup 10 --no-cpu-baseline" && \
timeout -k 10 600 bash scripts/gpu_pmc.sh r03zg_pmc_canonical
