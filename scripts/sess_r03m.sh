bash scripts/gpu_session.sh \
 "r03m_gputest:400:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "r03m_ab_canon:500:python scripts/variant_ab.py run 9 canonical"
