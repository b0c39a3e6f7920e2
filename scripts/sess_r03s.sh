bash scripts/gpu_session.sh \
 "r03s_ab_ragged_noreduce:500:python scripts/variant_ab.py run 5 ragged"
