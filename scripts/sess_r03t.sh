bash scripts/gpu_session.sh \
 "r03t_ab_canon_tailprio:500:python scripts/variant_ab.py run 7 canonical" \
 "r03t_ab_ragged_tailprio:500:python scripts/variant_ab.py run 5 ragged"
