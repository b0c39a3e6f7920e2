bash scripts/gpu_session.sh \
 "r03zt_gputest_stagger:400:WG_LANE_STAGGER=1 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ragged.py -q --timeout 250 --timeout-method thread" \
 "r03zt_k20_s0:200:python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-control" \
 "r03zt_k20_s1:200:WG_LANE_STAGGER=1 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-control" \
 "r03zt_k1000_s0:200:python bench.py --no-cpu-baseline --no-control" \
 "r03zt_k1000_s1:200:WG_LANE_STAGGER=1 python bench.py --no-cpu-baseline --no-control" \
 "r03zt_k20_s0b:200:python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-control" \
 "r03zt_k20_s1b:200:WG_LANE_STAGGER=1 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-control"
