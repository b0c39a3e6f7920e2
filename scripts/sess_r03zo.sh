T="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1"
bash scripts/gpu_session.sh \
 "r03zo_pipe_q8:300:GPU_MAX_HW_QUEUES=8 $T --master-port 29521 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-control" \
 "r03zo_serial_q8:300:GPU_MAX_HW_QUEUES=8 $T --master-port 29522 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-control --gather serial" \
 "r03zo_pipe_q4:300:$T --master-port 29523 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-control" \
 "r03zo_serial_q4:300:$T --master-port 29524 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-control --gather serial" \
 "r03zo_pipe_q8_k200:300:GPU_MAX_HW_QUEUES=8 $T --master-port 29525 bench.py --gpus 1 --steps 200 --warmup 5 --no-cpu-baseline --no-control" \
 "r03zo_serial_q4_k200:300:$T --master-port 29526 bench.py --gpus 1 --steps 200 --warmup 5 --no-cpu-baseline --no-control --gather serial"
