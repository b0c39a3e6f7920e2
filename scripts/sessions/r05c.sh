S=scripts/gpu_session.sh
W1="WORLD_SIZE=1,RANK=0,LOCAL_RANK=0,MASTER_ADDR=127.0.0.1,MASTER_PORT=29581"
$S "r05c_gputest_new:200:python -u -m pytest tests/test_gpu_prepared.py tests/test_gpu_policy_loop.py -x -q --timeout 120 --timeout-method thread" \
   "r05c_k20:900:KS='20 5' scripts/issue_ab.sh r05c 3 canonical plain:WG_BENCH_WARM_MS=0 plainw50:WG_BENCH_WARM_MS=50 plainw100:WG_BENCH_WARM_MS=100 plainw200:WG_BENCH_WARM_MS=200 w1w100:$W1,WG_BENCH_WARM_MS=100 w1lazy:$W1,WG_BENCH_LAZY_NCCL=1,WG_BENCH_WARM_MS=100 w1gloo:$W1,WG_DIST_BACKEND=gloo,WG_BENCH_WARM_MS=100" \
   "r05c_bal:600:KS='200 20;1000 100' BENCH_ARGS='--walkers 4096' scripts/issue_ab.sh r05c_bal 2 balance b0:WG_BENCH_WARM_MS=0 b100:WG_BENCH_WARM_MS=100"
