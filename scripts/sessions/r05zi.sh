S=scripts/gpu_session.sh
$S "r05zi_res_tests:400:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ragged.py tests/test_gpu_api.py -q -x --timeout 120 --timeout-method thread -k 'resident or rollout'" \
   "r05zi_ab_res_balance:400:WG_N=4096 WG_AB_RESIDENT=1 python scripts/variant_ab.py run 7 balance && cp gpurun_out/variant_ab_balance.json gpurun_out/r05zi_ab_resident_balance4096.json" \
   "r05zi_ab_res_canon:400:WG_AB_RESIDENT=1 python scripts/variant_ab.py run 5 canonical && cp gpurun_out/variant_ab_canonical.json gpurun_out/r05zi_ab_resident_canonical.json" \
   "r05zi_ab_res_balance65k:400:WG_N=65536 WG_AB_RESIDENT=1 python scripts/variant_ab.py run 5 balance && cp gpurun_out/variant_ab_balance.json gpurun_out/r05zi_ab_resident_balance65536.json"
