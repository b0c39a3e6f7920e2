bash scripts/gpu_session.sh \
 "r03g_step_overhead:200:python scripts/step_overhead.py canonical 65536" \
 "r03g_step_overhead_bal:200:python scripts/step_overhead.py balance 4096" \
 "r03g_plan_guard:200:python -u -m pytest tests/test_gpu_ragged.py -q -k out_of_cap --timeout 120 --timeout-method thread" \
 "r03g_stamps_bal:200:WG_WORKLOAD=balance WG_N=4096 WG_STAMPS_OUT=stamps_bal.json python scripts/stamps.py build_ablate/lib_stamps.so" \
 "r03g_bench_bal:200:python bench.py --workload balance --walkers 4096 --steps 200 --warmup 50 --no-cpu-baseline" \
 "r03g_bench_bal_kernarg:200:HIP_FORCE_DEV_KERNARG=1 python bench.py --workload balance --walkers 4096 --steps 200 --warmup 50 --no-cpu-baseline" \
 "r03g_pmc_chain_f64:200:WG_WORKLOAD=chain WG_N=4096 WG_STEPS=10 bash scripts/gpu_pmc.sh r03g_pmc_chain full" \
 "r03g_mix_ragged:200:WG_WORKLOAD=ragged bash scripts/gpu_pmc.sh r03g_pmcv_ragged valu"
