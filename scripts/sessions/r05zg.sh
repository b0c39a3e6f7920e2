S=scripts/gpu_session.sh
$S "r05zg_gputest:600:python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread" \
   "r05zg_smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
   "r05zg_bench_k20:200:python bench.py --gpus 1 --steps 20 --warmup 5" \
   "r05zg_torchrun1:240:python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29651 bench.py --gpus 1 --steps 20 --warmup 5"
