#!/usr/bin/env python3
"""Per-step timeline right after the process group comes up (profiling aid, not product).  Launched as one rank:

    python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 --master-port P scripts/rccl_warm.py

Builds the bench's canonical env, runs W warm-up steps (as bench.py does, before the group), brings up the group
(WG_DIST_BACKEND: nccl = RCCL, or gloo), barriers, then times S steps one by one with HIP events on the env's calling
stream and prints the per-step series (median of blocks of 10): what the first steps after the group's
initialisation cost against the steady state.  gpurun_out/rccl_warm_<backend>.json."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from bench import make_spec  # noqa: E402
from walker_gym_amd.batched_env import BatchedPhysicsEnv  # noqa: E402

backend = os.environ.get("WG_DIST_BACKEND", "nccl")
W, S = int(os.environ.get("WG_W", "5")), int(os.environ.get("WG_S", "300"))
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
N = 65536
spec, params = make_spec("canonical", N, seed=1000)
env = BatchedPhysicsEnv(spec, device=dev, **params)
env.reserve_streams(2)
acts = (torch.rand((max(W, 1), N, 8), device=dev) * 2 - 1).contiguous()
acts_t = (torch.rand((S, N, 8), device=dev) * 2 - 1).contiguous()
env.run(acts, W, lanes=2)
torch.cuda.synchronize()
t0 = time.perf_counter()
if backend == "nccl":
    dist.init_process_group("nccl", device_id=dev)
elif backend != "none":
    dist.init_process_group(backend)
init_s = time.perf_counter() - t0
if backend != "none":
    dist.barrier()
torch.cuda.synchronize()
idle_s = time.perf_counter() - t0
stream = torch.cuda.current_stream(dev)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(S + 1)]
ev[0].record(stream)
for s in range(S):
    env.run(acts_t[s:s + 1].contiguous(), 1, lanes=2)
    ev[s + 1].record(stream)
torch.cuda.synchronize()
us = [ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(S)]
blocks = [round(sorted(us[i:i + 10])[5], 2) for i in range(0, S, 10)]
out = {"backend": backend, "warmup": W, "steps": S, "group_init_s": round(init_s, 3), "gpu_idle_s": round(idle_s, 3),
       "us_per_step_blocks_of_10_median": blocks, "first_20_mean": round(sum(us[:20]) / 20, 2),
       "last_100_mean": round(sum(us[-100:]) / 100, 2)}
print(json.dumps(out))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", f"rccl_warm_{backend}_w{W}.json"), "w"), indent=1)
if backend != "none":
    dist.destroy_process_group()
