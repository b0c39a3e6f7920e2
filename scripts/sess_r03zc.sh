bash scripts/gpu_session.sh \
 "r03zc_bench:300:python bench.py --resident" \
 "r03zc_prof_canonical:300:rocprofv3 --kernel-trace --stats -d gpurun_out/r03zc_prof_canonical -o run --output-format csv -- python bench.py --no-cpu-baseline" \
 "r03zc_bench_ragged:300:python bench.py --workload ragged --no-cpu-baseline" \
 "r03zc_ab_canon:500:python scripts/variant_ab.py run 5 canonical"
