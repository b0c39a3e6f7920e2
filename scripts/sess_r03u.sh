bash scripts/gpu_session.sh \
 "r03u_gputest:500:python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread" \
 "r03u_ab_chain:500:WG_N=4096 python scripts/variant_ab.py run 5 chain" \
 "r03u_ab_perfdemo:500:WG_N=4096 python scripts/variant_ab.py run 5 perfdemo"
