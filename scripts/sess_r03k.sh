bash scripts/gpu_session.sh \
 "r03k_ab_ragged:600:python scripts/variant_ab.py run 5 ragged"
