bash scripts/gpu_session.sh \
 "r03p_ab_ragged:500:python scripts/variant_ab.py run 7 ragged" \
 "r03p_ab_canon:500:python scripts/variant_ab.py run 7 canonical"
