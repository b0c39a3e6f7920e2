#!/usr/bin/env python3
"""Minimal driver for rocprofv3 PMC passes: N canonical walkers, W warmup + S timed steps."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from walker_gym_amd.batched_env import BatchedPhysicsEnv  # noqa: E402
from walker_gym_amd.synthetic import canonical_walkers  # noqa: E402

n = int(os.environ.get("WG_N", "65536"))
steps = int(os.environ.get("WG_STEPS", "30"))
env = BatchedPhysicsEnv(canonical_walkers(n, seed=0), in3d=1)
acts = (torch.rand((steps, n, 8), device="cuda") * 2 - 1).contiguous()
env.run(acts, steps, lanes=1)   # one full-batch launch per step: PMC values per dispatch = per step
torch.cuda.synchronize()
print("done", steps, "steps")
