S=scripts/gpu_session.sh
W1="WORLD_SIZE=1,RANK=0,LOCAL_RANK=0,MASTER_ADDR=127.0.0.1,MASTER_PORT=29571"
$S "r05b_gputest:300:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
   "r05b_ab_canonical:400:python scripts/variant_ab.py run 5 canonical && cp gpurun_out/variant_ab_canonical.json gpurun_out/r05b_ab_canonical.json" \
   "r05b_ab_ragged:400:python scripts/variant_ab.py run 5 ragged && cp gpurun_out/variant_ab_ragged.json gpurun_out/r05b_ab_ragged.json" \
   "r05b_ab_balance:300:WG_N=4096 python scripts/variant_ab.py run 7 balance && cp gpurun_out/variant_ab_balance.json gpurun_out/r05b_ab_balance.json" \
   "r05b_k20:600:KS='20 5' scripts/issue_ab.sh r05b 4 canonical plain:WG_BENCH_WARM_MS=0 plainw20:WG_BENCH_WARM_MS=20 w1:$W1,WG_BENCH_WARM_MS=0 w1w20:$W1,WG_BENCH_WARM_MS=20 w1w100:$W1,WG_BENCH_WARM_MS=100"
