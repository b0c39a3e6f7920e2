bash scripts/gpu_session.sh \
 "r03zn_gputest_dist:300:python -u -m pytest tests/test_gpu_distributed.py -x -q --timeout 250 --timeout-method thread" \
 "r03zn_bench_nccl1_k20_pipe:300:python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline" \
 "r03zn_bench_nccl1_k20_serial:300:python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --gather serial" \
 "r03zn_bench_nccl1:300:python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 1 --no-cpu-baseline" \
 "r03zn_rehearsal_gloo2_k20:300:WG_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29514 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline"
