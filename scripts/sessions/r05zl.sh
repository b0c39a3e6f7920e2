S=scripts/gpu_session.sh
$S "r05zl_bench_default:400:python bench.py" "r05zl_bench_driver:300:python bench.py --gpus 1 --steps 20 --warmup 5"
