bash scripts/gpu_session.sh \
 "r03zh_ab_hist_canonical:400:python scripts/variant_ab.py run 5 canonical" \
 "r03zh_ab_hist_ragged:400:python scripts/variant_ab.py run 5 ragged" \
 "r03zh_ab_hist_balance4096:300:WG_N=4096 python scripts/variant_ab.py run 5 balance"
