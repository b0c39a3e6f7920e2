"""In-process A/B: BatchedPhysicsEnv.run (one C call per walker range) vs the same steps captured into a HIP
graph and replayed, on the canonical bench workload.  usage: python scripts/graph_ab.py [rounds]"""
import statistics
import sys

import torch

sys.path.insert(0, ".")
from bench import make_spec  # noqa: E402
from walker_gym_amd.batched_env import BatchedPhysicsEnv  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
N, S = 65536, 200
spec, params = make_spec("canonical", N, seed=1000)
env = BatchedPhysicsEnv(spec, device="cuda:0", **params)
acts = (torch.rand((S, N, env.batch.A), device="cuda:0") * 2 - 1).contiguous()
g = env.graph(acts, S)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
res = {"run": [], "graph": []}
env.run(acts, S)
for r in range(rounds):
    for k in res:
        e0.record()
        if k == "run":
            env.run(acts, S)
        else:
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        res[k].append(e0.elapsed_time(e1) / S * 1e3)
    print(f"round {r}: " + "  ".join(f"{k} {v[-1]:.1f}" for k, v in res.items()), flush=True)
for k, v in res.items():
    print(f"{k:6s} median {statistics.median(v):6.1f} us  min {min(v):6.1f} us", flush=True)
