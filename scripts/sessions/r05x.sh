S=scripts/gpu_session.sh
$S "r05x_stamps_bal:200:WG_N=4096 WG_WORKLOAD=balance WG_STAMPS_OUT=r05x_stamps_balance4096.json python scripts/stamps.py" \
   "r05x_stamps_canon:200:WG_STAMPS_OUT=r05x_stamps_canonical.json python scripts/stamps.py" \
   "r05x_gloo2:300:WG_DIST_BACKEND=gloo python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline --no-control" \
   "r05x_nccl1:240:python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29641 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-control" \
   "r05x_ab_wpw:300:WG_N=4096 WG_AB_ONLY=none python scripts/variant_ab.py run 7 balance w8: w4:WG_LEAN_WPW=4 w2:WG_LEAN_WPW=2 && cp gpurun_out/variant_ab_balance.json gpurun_out/r05x_ab_wpw_balance4096.json" \
   "r05x_policy_tests:300:python -u -m pytest tests/test_gpu_policy_loop.py -q -x --timeout 120 --timeout-method thread" \
   "r05x_bench_pol:300:python bench.py --no-cpu-baseline" \
   "r05x_bench_pol_ragged:300:python bench.py --workload ragged --no-cpu-baseline"
