S=scripts/gpu_session.sh
$S "r05x_stamps_bal:200:WG_N=4096 WG_WORKLOAD=balance WG_STAMPS_OUT=r05x_stamps_balance4096.json python scripts/stamps.py" \
   "r05x_stamps_canon:200:WG_STAMPS_OUT=r05x_stamps_canonical.json python scripts/stamps.py" \
   "r05x_gloo2:300:WG_DIST_BACKEND=gloo python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline --no-control"
$S "r05x_nccl1:240:python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29641 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-control"
