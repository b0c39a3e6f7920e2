bash scripts/gpu_session.sh \
 "r03d_gputest:600:python -u -m pytest tests -m gpu -q --timeout 250 --timeout-method thread" \
 "r03d_bench:240:python bench.py" \
 "r03d_valu_peak:60:./build_ablate/valu_peak" \
 "r03d_launch_floor:60:./build_ablate/launch_floor" \
 "r03d_ab_ragged:300:python scripts/variant_ab.py run 3 ragged base:WG_TILE_WINDOW=0,WG_XCD=0 win:WG_TILE_WINDOW=512,WG_XCD=0 xcd:WG_TILE_WINDOW=0,WG_XCD=1 both:WG_TILE_WINDOW=512,WG_XCD=1" \
 "r03d_pmc_ragged:200:WG_WORKLOAD=ragged bash scripts/gpu_pmc.sh r03d_pmc_ragged" \
 "r03d_bench_ragged:240:python bench.py --workload ragged --no-cpu-baseline" \
 "r03d_bench_chain:240:python bench.py --workload chain --walkers 4096 --chain-points 100 --steps 100 --warmup 10 --cpu-seconds 8" \
 "r03d_bench_perfdemo:240:python bench.py --workload perfdemo --walkers 4096 --chain-points 100 --steps 100 --warmup 10 --cpu-seconds 8" \
 "r03d_bench_balance4096:200:python bench.py --workload balance --walkers 4096 --graph --steps 1000 --warmup 100 --no-cpu-baseline" \
 "r03d_pmc_mix:300:bash scripts/gpu_pmc_mix.sh r03d_mix base abl1 abl2 abl16"
