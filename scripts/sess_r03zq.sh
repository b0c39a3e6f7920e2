bash scripts/gpu_session.sh \
 "r03zq_ab_sqinl_balance4096:300:WG_N=4096 python scripts/variant_ab.py run 9 balance" \
 "r03zq_ab_sqinl_canonical:400:python scripts/variant_ab.py run 5 canonical" \
 "r03zq_ab_sqinl_ragged:400:python scripts/variant_ab.py run 5 ragged"
