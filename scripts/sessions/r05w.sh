# round-5 final measurement session at HEAD (after ABI 12 and the communicator-after-the-clock bench): the r05m
# session (GPU suite, smoke, every bench line, rocprofv3 traces, PMC) plus the K = 20 plain / world-1 kernel traces
W1="WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29571"
TAG=r05w bash scripts/sessions/r05m.sh && \
scripts/gpu_session.sh \
   "r05w_trace_k20_plain:180:rocprofv3 --kernel-trace --stats -d gpurun_out/r05w_trace_k20_plain -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-control" \
   "r05w_trace_k20_world1:180:export $W1; rocprofv3 --kernel-trace --stats -d gpurun_out/r05w_trace_k20_world1 -o run --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-control"
