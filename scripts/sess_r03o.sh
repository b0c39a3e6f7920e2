bash scripts/gpu_session.sh \
 "r03o_bench:300:python bench.py --resident" \
 "r03o_prof_canonical:300:rocprofv3 --kernel-trace --stats -d gpurun_out/r03o_prof_canonical -o run --output-format csv -- python bench.py --no-cpu-baseline" \
 "r03o_pmc_canonical:200:bash scripts/gpu_pmc.sh r03o_pmc_canonical" \
 "r03o_bench_ragged:300:python bench.py --workload ragged --no-cpu-baseline" \
 "r03o_prof_ragged:300:rocprofv3 --kernel-trace --stats -d gpurun_out/r03o_prof_ragged -o run --output-format csv -- python bench.py --workload ragged --no-cpu-baseline" \
 "r03o_bench_balance4096:200:python bench.py --workload balance --walkers 4096 --graph --steps 1000 --warmup 100 --no-cpu-baseline"
