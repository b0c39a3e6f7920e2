S=scripts/gpu_session.sh
$S "r05zb_gputest:600:python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread" \
   "r05zb_smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'"
