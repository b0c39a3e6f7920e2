S=scripts/gpu_session.sh
$S "r05n_gputest_pl:300:python -u -m pytest tests/test_gpu_policy_loop.py tests/test_gpu_prepared.py -q --timeout 120 --timeout-method thread" \
   "r05n_bench_ragged:400:python bench.py --workload ragged --no-cpu-baseline"
