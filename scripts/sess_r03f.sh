bash scripts/gpu_session.sh \
 "r03f_gputest:600:python -u -m pytest tests -m gpu -q --timeout 250 --timeout-method thread" \
 "r03f_bench:240:python bench.py --resident" \
 "r03f_prof_canonical:240:rocprofv3 --kernel-trace --stats -d gpurun_out/r03f_prof_canonical -o run --output-format csv -- python bench.py --no-cpu-baseline" \
 "r03f_pmc_canonical:200:bash scripts/gpu_pmc.sh r03f_pmc_canonical" \
 "r03f_bench_ragged:240:python bench.py --workload ragged --no-cpu-baseline" \
 "r03f_prof_ragged:240:rocprofv3 --kernel-trace --stats -d gpurun_out/r03f_prof_ragged -o run --output-format csv -- python bench.py --workload ragged --no-cpu-baseline" \
 "r03f_bench_balance4096:200:python bench.py --workload balance --walkers 4096 --graph --steps 1000 --warmup 100 --no-cpu-baseline"
