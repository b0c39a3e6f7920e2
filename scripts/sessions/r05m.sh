# round-5 measurement session at HEAD: GPU suite, smoke, every bench line, rocprofv3 traces, PMC traffic passes
S=scripts/gpu_session.sh
t=${TAG:-r05m}
$S "${t}_gputest:300:python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread" \
   "${t}_smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
   "${t}_bench_k20:180:python bench.py --gpus 1 --steps 20 --warmup 5" \
   "${t}_bench_k20b:180:python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline" \
   "${t}_bench:300:python bench.py --resident" \
   "${t}_prof_canonical:300:rocprofv3 --kernel-trace --stats -d gpurun_out/${t}_prof_canonical -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 200" \
   "${t}_bench_ragged:400:python bench.py --workload ragged" \
   "${t}_prof_ragged:300:rocprofv3 --kernel-trace --stats -d gpurun_out/${t}_prof_ragged -o run --output-format csv -- python bench.py --workload ragged --no-cpu-baseline --steps 200" \
   "${t}_bench_balance4096:300:python bench.py --workload balance --walkers 4096 --graph --resident --steps 1000 --warmup 100" \
   "${t}_bench_chain:400:python bench.py --workload chain --walkers 4096 --chain-points 100 --steps 100 --warmup 10 --cpu-seconds 10" \
   "${t}_bench_perfdemo:400:python bench.py --workload perfdemo --walkers 4096 --chain-points 100 --steps 100 --warmup 10 --cpu-seconds 10" \
   "${t}_nccl1:240:python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29631 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline" \
   "${t}_pmc:400:bash scripts/gpu_pmc.sh ${t}_pmc_canonical && WG_WORKLOAD=ragged bash scripts/gpu_pmc.sh ${t}_pmc_ragged"
