bash scripts/gpu_session.sh \
 "r03zl_stamps_balance4096:200:WG_N=4096 WG_WORKLOAD=balance python scripts/stamps.py build_ab/lib_stamps.so && cp gpurun_out/stamps.json gpurun_out/r03zl_stamps_balance4096.json" \
 "r03zl_stamps_canonical:200:python scripts/stamps.py build_ab/lib_stamps.so && cp gpurun_out/stamps.json gpurun_out/r03zl_stamps_canonical.json"
