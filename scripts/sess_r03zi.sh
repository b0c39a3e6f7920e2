bash scripts/gpu_session.sh \
 "r03zi_ab_guards_balance4096:400:WG_N=4096 python scripts/variant_ab.py run 7 balance"
