mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "lanes" -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_lanes.log 2>&1 || { tail -30 gpurun_out/pytest_lanes.log; exit 1; }
tail -3 gpurun_out/pytest_lanes.log
for L in 1 2 3; do WG_LANES=$L timeout -k 10 120 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-control --workload ragged > gpurun_out/rag_$L.log 2>&1 || exit 1; grep -o '"ms_per_step": [0-9.]*' gpurun_out/rag_$L.log; done
