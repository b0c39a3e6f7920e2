bash scripts/gpu_session.sh \
 "r03l_gputest_ragged:300:python -u -m pytest tests/test_gpu_ragged.py tests/test_gpu_parity.py tests/test_gpu_api.py -m gpu -x -q --timeout 120 --timeout-method thread" \
 "r03l_ab_ragged:500:python scripts/variant_ab.py run 7 ragged"
