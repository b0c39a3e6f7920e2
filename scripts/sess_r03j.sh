bash scripts/gpu_session.sh \
 "r03j_stamps_canon:200:WG_STAMPS_OUT=r03j_stamps_canon.json python scripts/stamps.py build_ablate/lib_stamps.so" \
 "r03j_stamps_ragged:200:WG_WORKLOAD=ragged WG_STAMPS_OUT=r03j_stamps_ragged.json python scripts/stamps.py build_ablate/lib_stamps.so"
