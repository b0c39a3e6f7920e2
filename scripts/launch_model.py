#!/usr/bin/env python3
"""Per-launch time of the canonical step against batch size, one full-batch launch per step (lanes 1), HIP events
over 200 launches after 30 warm-up (profiling aid, not product).  A launch is modelled as T(N) = a + b*N: b is the
throughput cost per walker, a the fixed cost of a launch (the ramp while the first round's loads land, the drain
while the last round computes).  usage: launch_model.py [N ...]; env variants via the environment (WG_*)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from walker_gym_amd.batched_env import BatchedPhysicsEnv  # noqa: E402
from walker_gym_amd.synthetic import canonical_walkers  # noqa: E402

Ns = [int(a) for a in sys.argv[1:]] or [8192, 16384, 32768, 49152, 65536, 98304, 131072]
steps, res = 200, {}
for n in Ns:
    env = BatchedPhysicsEnv(canonical_walkers(n, seed=0), in3d=1)
    acts = (torch.rand((steps, n, 8), device="cuda") * 2 - 1).contiguous()
    env.run(acts[:30].contiguous(), 30, lanes=1)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); env.run(acts, steps, lanes=1); e1.record(); torch.cuda.synchronize()
    res[n] = e0.elapsed_time(e1) / steps * 1e3
    print(f"N={n:7d} {res[n]:8.2f} us/launch", flush=True)
    del env, acts
x = np.array(list(res), float); y = np.array(list(res.values()))
b, a = np.polyfit(x, y, 1)
out = {"us_per_launch": res, "fit_a_us": round(float(a), 3), "fit_b_us_per_65536": round(float(b) * 65536, 3),
       "env": {k: v for k, v in os.environ.items() if k.startswith("WG_")}}
print(json.dumps(out), flush=True)
