bash scripts/gpu_session.sh \
 "r03h_inst_rate:120:./build_ablate/inst_rate" \
 "r03h_bench:300:python bench.py --steps 300 --warmup 50 --no-cpu-baseline"
