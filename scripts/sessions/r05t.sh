S=scripts/gpu_session.sh
W1="WORLD_SIZE=1,RANK=0,LOCAL_RANK=0,MASTER_ADDR=127.0.0.1,MASTER_PORT=29631"
$S "r05t_torchrun1:300:python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29633 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05t_torchrun1.json" \
   "r05t_k20:900:KS='20 5;1000 50' scripts/issue_ab.sh r05t 3 canonical plain: w1lazy:$W1 w1eager:$W1,WG_COMM_EAGER=1"
