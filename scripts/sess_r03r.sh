bash scripts/gpu_session.sh \
 "r03r_ab_ragged_hop:500:python scripts/variant_ab.py run 7 ragged"
