bash scripts/gpu_session.sh \
 "r03n_gputest:400:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "r03n_ab_canon:500:python scripts/variant_ab.py run 9 canonical" \
 "r03n_ab_bal:300:WG_N=4096 python scripts/variant_ab.py run 9 balance"
