"""In-process A/B on the ragged bench workload (65,536 mixed walkers): WG_LEAN_PRIO 0 / 1 (the workgroup
kernel's load-phase priority) x 1 / 2 plan-block ranges.  usage: python scripts/ragged_ab.py [rounds]"""
import os
import statistics
import sys

import torch

sys.path.insert(0, ".")
from bench import make_spec  # noqa: E402
from walker_gym_amd.batched_env import BatchedPhysicsEnv  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
N, S = 65536, 100
spec, params = make_spec("ragged", N, seed=1000)
env = BatchedPhysicsEnv(spec, device="cuda:0", **params)
acts = (torch.rand((S, N, env.batch.A), device="cuda:0") * 2 - 1).contiguous()
V = {"p1_L2": ("1", "2"), "p0_L2": ("0", "2"), "p1_L1": ("1", "1"), "p0_L1": ("0", "1")}
res = {k: [] for k in V}
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for r in range(rounds):
    for k, (pr, ln) in V.items():
        os.environ["WG_LEAN_PRIO"], os.environ["WG_LANES"] = pr, ln
        env.run(acts[:10], 10)
        e0.record()
        env.run(acts, S)
        e1.record()
        torch.cuda.synchronize()
        res[k].append(e0.elapsed_time(e1) / S * 1e3)
    print(f"round {r}: " + "  ".join(f"{k} {v[-1]:.1f}" for k, v in res.items()), flush=True)
for k, v in res.items():
    print(f"{k:6s} median {statistics.median(v):6.1f} us  min {min(v):6.1f} us", flush=True)
