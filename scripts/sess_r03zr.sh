bash scripts/gpu_session.sh \
 "r03zr_gputest:500:python -u -m pytest tests -m gpu -q --timeout 250 --timeout-method thread" \
 "r03zr_ab_ne1inl_balance4096:300:WG_N=4096 python scripts/variant_ab.py run 9 balance" \
 "r03zr_ab_ne1inl_canonical:400:python scripts/variant_ab.py run 5 canonical"
