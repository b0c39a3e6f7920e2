#!/usr/bin/env python3
"""Per-launch time of the canonical step vs batch size (fixed launch overhead = 2*T(N) - T(2N))."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from walker_gym_amd.batched_env import BatchedPhysicsEnv  # noqa: E402
from walker_gym_amd.synthetic import canonical_walkers  # noqa: E402

for n in [int(a) for a in sys.argv[1:]] or [16384, 32768, 65536, 131072, 262144]:
    steps = 100
    env = BatchedPhysicsEnv(canonical_walkers(n, seed=0), in3d=1)
    acts = (torch.rand((steps, n, 8), device="cuda") * 2 - 1).contiguous()
    env.run(acts[:10].contiguous(), 10)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); env.run(acts, steps); e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / steps * 1e3
    print(f"N={n:7d} {us:8.1f} us/step  {us / n * 1e3:6.3f} ns/walker", flush=True)
    del env, acts
