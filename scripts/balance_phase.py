#!/usr/bin/env python3
"""Config 2 (4,096 Balance-v0 walkers) per-step time along a long rollout, beside the number of walkers whose state has
gone non-finite (the reference's Balance-v0 diverges under U(-1, 1) actions: ~3 % of walkers by step 1,000, from step
~350, as gym/optimized_walker.py's creature does; the kernel then runs those walkers' waves through the exact IEEE cold
paths).  Windows of W steps, one prepared launch per step (lanes 1), HIP events; actions U(-s, s) for each scale s.
    python scripts/balance_phase.py [steps=1500] [window=100] [scales=1,0]  -> gpurun_out/balance_phase.json"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import make_spec  # noqa: E402
from walker_gym_amd.batched_env import BatchedPhysicsEnv  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 1500
    win = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    scales = [float(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "1,0").split(",")]
    n = int(os.environ.get("WG_N", "4096"))
    workload = os.environ.get("WG_WORKLOAD", "balance")   # (any bench.py workload: ragged for config 5)
    out = {"workload": workload, "walkers": n, "window": win, "runs": {}}
    for s in scales:
        spec, params = make_spec(workload, n, seed=1000)
        env = BatchedPhysicsEnv(spec, device="cuda:0", **params)
        g = torch.Generator(device="cuda:0").manual_seed(7)
        acts = ((torch.rand((steps, n, env.batch.A), generator=g, device="cuda:0") * 2 - 1) * s).contiguous()
        rows = []
        wpw = env.launch_geometry()["walkers_per_block"]   # (-1 for wave tiles: walkers per wave vary)
        wid = torch.as_tensor(np.repeat(np.arange(n), np.diff(np.asarray(spec["mass_off"]))), device="cuda:0")
        for w0 in range(0, steps, win):
            prep = env.prepare_run(acts[w0:w0 + win], win, lanes=1)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            prep()
            e1.record()
            torch.cuda.synchronize()
            badm = (~torch.isfinite(env.pos).all(1)).int()
            bad = torch.zeros(n, dtype=torch.int32, device="cuda:0").index_put_((wid,), badm, accumulate=True) > 0
            waves = bad.reshape(-1, wpw).any(1) if wpw > 0 and n % wpw == 0 else bad
            rows.append({"steps": [w0, w0 + win], "us_per_step": round(e0.elapsed_time(e1) / win * 1e3, 3),
                         "nonfinite_walkers": int(bad.sum()), "waves_with_nonfinite": int(waves.sum()),
                         "waves": int(waves.numel())})
            print(s, rows[-1], flush=True)
        out["runs"][str(s)] = rows
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "balance_phase.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
