S=scripts/gpu_session.sh
$S "r05zk_graph_tests:300:python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -k 'graph'"
