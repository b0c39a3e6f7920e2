bash scripts/gpu_session.sh \
 "r03zf_gputest_ragged:300:python -u -m pytest tests/test_gpu_ragged.py -x -q --timeout 200 --timeout-method thread" \
 "r03zf_ab_dual_sum:500:python scripts/variant_ab.py run 7 ragged"
