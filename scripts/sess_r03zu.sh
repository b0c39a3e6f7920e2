bash scripts/gpu_session.sh \
 "r03zu_gputest:500:python -u -m pytest tests -m gpu -q --timeout 250 --timeout-method thread" \
 "r03zu_smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'"
