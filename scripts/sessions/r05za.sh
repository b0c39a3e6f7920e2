S=scripts/gpu_session.sh
$S "r05za_bench:300:python bench.py --no-cpu-baseline" \
   "r05za_bench_ragged:300:python bench.py --workload ragged --no-cpu-baseline" \
   "r05za_bench_balance:300:python bench.py --workload balance --walkers 4096 --graph --resident --steps 1000 --warmup 100 --no-cpu-baseline" \
   "r05za_valu:400:bash scripts/gpu_pmc.sh r05za_valu_canonical valu && WG_WORKLOAD=ragged bash scripts/gpu_pmc.sh r05za_valu_ragged valu"
