bash scripts/gpu_session.sh \
 "r03zs_smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "r03zs_bench:300:python bench.py --resident" \
 "r03zs_bench_balance4096:200:python bench.py --workload balance --walkers 4096 --graph --steps 1000 --warmup 100 --no-cpu-baseline" \
 "r03zs_bench_ragged:300:python bench.py --workload ragged --no-cpu-baseline" \
 "r03zs_prof_canonical:300:rocprofv3 --kernel-trace --stats -d gpurun_out/r03zs_prof_canonical -o run --output-format csv -- python bench.py --no-cpu-baseline"
