#!/usr/bin/env python3
"""Minimal driver for rocprofv3 PMC passes: WG_N walkers of bench.py's WG_WORKLOAD (default canonical), WG_STEPS
steps, one full-batch launch per step (lanes 1), so per-dispatch PMC values are per step."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench import make_spec  # noqa: E402
from walker_gym_amd.batched_env import BatchedPhysicsEnv  # noqa: E402

n = int(os.environ.get("WG_N", "65536"))
steps = int(os.environ.get("WG_STEPS", "30"))
workload = os.environ.get("WG_WORKLOAD", "canonical")
spec, params = make_spec(workload, n, seed=1000)
env = BatchedPhysicsEnv(spec, **params)
acts = (torch.rand((steps, n, max(1, env.batch.A)), device="cuda") * 2 - 1).contiguous()
env.run(acts, steps, lanes=1)
torch.cuda.synchronize()
print("done", workload, steps, "steps")
