bash scripts/gpu_session.sh \
 "r03zm_gputest:400:python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread" \
 "r03zm_ab_norm_balance4096:300:WG_N=4096 python scripts/variant_ab.py run 7 balance" \
 "r03zm_ab_norm_canonical:400:python scripts/variant_ab.py run 5 canonical"
