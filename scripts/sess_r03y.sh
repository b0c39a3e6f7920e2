bash scripts/gpu_session.sh \
 "r03y_gputest:500:python -u -m pytest tests -m gpu -q --timeout 250 --timeout-method thread" \
 "r03y_ab_canon:500:python scripts/variant_ab.py run 7 canonical" \
 "r03y_ab_ragged:500:python scripts/variant_ab.py run 5 ragged" \
 "r03y_ab_perfdemo:500:WG_N=4096 python scripts/variant_ab.py run 3 perfdemo"
