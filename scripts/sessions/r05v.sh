S=scripts/gpu_session.sh
$S "r05v_gputest_pairs:400:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ragged.py -q -x --timeout 120 --timeout-method thread -k 'pair or golden or bit_exact'" \
   "r05v_ab_stagger:600:python scripts/variant_ab.py run 5 canonical && cp gpurun_out/variant_ab_canonical.json gpurun_out/r05v_ab_stagger_canonical.json"
