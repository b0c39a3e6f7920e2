S=scripts/gpu_session.sh
$S "r05o_fullsize:400:python -u -m pytest tests/test_gpu_parity.py::test_full_size_vs_oracle tests/test_gpu_ragged.py::test_full_size_ragged_vs_oracle -q --timeout 300 --timeout-method thread" \
   "r05o_stamps_bal:200:WG_N=4096 WG_WORKLOAD=balance WG_STAMPS_OUT=r05o_stamps_balance4096.json python scripts/stamps.py"
