bash scripts/gpu_session.sh \
 "r03i_gputest:400:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "r03i_ab_canon:400:python scripts/variant_ab.py run 7 canonical" \
 "r03i_ab_ragged:400:python scripts/variant_ab.py run 5 ragged"
