bash scripts/gpu_session.sh \
 "r03z_gputest:500:python -u -m pytest tests -m gpu -q --timeout 250 --timeout-method thread" \
 "r03z_ab_canon:500:python scripts/variant_ab.py run 7 canonical" \
 "r03z_ab_ragged:500:python scripts/variant_ab.py run 5 ragged" \
 "r03z_ab_canon_res:400:WG_AB_RESIDENT=1 python scripts/variant_ab.py run 3 canonical"
