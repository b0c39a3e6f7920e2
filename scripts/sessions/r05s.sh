S=scripts/gpu_session.sh
$S "r05s_gputest:600:python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread" \
   "r05s_ab_inc8_canonical:400:WG_AB_ONLY=none python scripts/variant_ab.py run 5 canonical i8:WG_INC8=1 i16:WG_INC8=0 && cp gpurun_out/variant_ab_canonical.json gpurun_out/r05s_ab_inc8_canonical.json" \
   "r05s_ab_inc8_ragged:400:WG_AB_ONLY=none python scripts/variant_ab.py run 5 ragged i8:WG_INC8=1 i16:WG_INC8=0 && cp gpurun_out/variant_ab_ragged.json gpurun_out/r05s_ab_inc8_ragged.json" \
   "r05s_ab_inc8_balance:300:WG_N=4096 WG_AB_ONLY=none python scripts/variant_ab.py run 5 balance i8:WG_INC8=1 i16:WG_INC8=0 && cp gpurun_out/variant_ab_balance.json gpurun_out/r05s_ab_inc8_balance4096.json" \
   "r05s_bench_inc8:500:KS='20 5;1000 50' scripts/issue_ab.sh r05s 3 canonical i8:WG_INC8=1 i16:WG_INC8=0"
