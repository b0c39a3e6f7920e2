bash scripts/gpu_session.sh \
 "r03v_ab_chain:600:WG_N=4096 python scripts/variant_ab.py run 5 chain" \
 "r03v_ab_perfdemo:600:WG_N=4096 python scripts/variant_ab.py run 5 perfdemo"
