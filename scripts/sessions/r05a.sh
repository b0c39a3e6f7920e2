S=scripts/gpu_session.sh
W1="WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29561"
$S "r05a_gputest:300:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
   "r05a_ab_balance:300:WG_N=4096 python scripts/variant_ab.py run 7 balance" \
   "r05a_bench_balance4096:240:python bench.py --workload balance --walkers 4096 --graph --resident --steps 1000 --warmup 100 --cpu-seconds 5" \
   "r05a_k20_plain1:120:python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-control" \
   "r05a_k20_world1a:120:env $W1 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-control" \
   "r05a_k20_plain2:120:python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-control" \
   "r05a_k20_torchrun:150:python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29562 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-control" \
   "r05a_k20_world1b:120:env $W1 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-control" \
   "r05a_trace_k20_plain:180:rocprofv3 --kernel-trace --stats -d gpurun_out/r05a_trace_k20_plain -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-control" \
   "r05a_trace_k20_world1:180:export $W1; rocprofv3 --kernel-trace --stats -d gpurun_out/r05a_trace_k20_world1 -o run --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-control" \
   "r05a_bench:300:python bench.py --resident --cpu-seconds 8"
