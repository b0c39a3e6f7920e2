bash scripts/gpu_session.sh \
 "r03zj_ab_zm_balance4096:400:WG_N=4096 python scripts/variant_ab.py run 7 balance wpw4:WG_LEAN_WPW=4 wpw2:WG_LEAN_WPW=2" \
 "r03zj_ab_zm_canonical:400:python scripts/variant_ab.py run 5 canonical"
