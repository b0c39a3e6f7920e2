S=scripts/gpu_session.sh
$S "r05zm_ab_bal:500:WG_N=4096 python scripts/variant_ab.py run 9 balance && cp gpurun_out/variant_ab_balance.json gpurun_out/r05zm_ab_noxcd1_balance4096.json" \
   "r05zm_ab_bal65k:400:WG_N=65536 python scripts/variant_ab.py run 5 balance && cp gpurun_out/variant_ab_balance.json gpurun_out/r05zm_ab_noxcd1_balance65536.json"
